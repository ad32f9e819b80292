"""Pure-Python emulation of the neighbour *set* CPU ``torch.topk`` returns (TEST INFRA ONLY).

``simulator.py:19`` calls ``torch.topk(dist, k, largest=False)``.  On CPU, for
``k*64 > n`` torch's TopKImpl builds ``queue[j] = (value_j, j)`` and calls
``std::nth_element(queue.begin(), queue.begin()+k-1, queue.end(), comp)`` with
``comp(x, y) = x.first < y.first`` (no index tie-break), then keeps the first
k entries.  Which indices survive when distances tie at the k-boundary is
therefore decided by libstdc++'s introselect:

  __introselect(depth = 2*floor(log2 n)): while len > 3 { depth==0 -> heap_select;
  median-of-3 to first (a=first+1, b=mid, c=last-1), unguarded partition } then
  insertion sort.

The HIP kernel (``csrc/swarm_knn.h``) runs the same steps per row; this module
is the readable restatement it is tested against, and it is itself pinned to
torch.topk by ``tests/golden/topk_ties.npz``.
"""
from __future__ import annotations


def _lt(x, y):
    return x[0] < y[0]


def _move_median_to_first(a, result, x, y, z):
    if _lt(a[x], a[y]):
        if _lt(a[y], a[z]):
            a[result], a[y] = a[y], a[result]
        elif _lt(a[x], a[z]):
            a[result], a[z] = a[z], a[result]
        else:
            a[result], a[x] = a[x], a[result]
    elif _lt(a[x], a[z]):
        a[result], a[x] = a[x], a[result]
    elif _lt(a[y], a[z]):
        a[result], a[z] = a[z], a[result]
    else:
        a[result], a[y] = a[y], a[result]


def _unguarded_partition(a, first, last, pivot):
    while True:
        while _lt(a[first], a[pivot]):
            first += 1
        last -= 1
        while _lt(a[pivot], a[last]):
            last -= 1
        if not first < last:
            return first
        a[first], a[last] = a[last], a[first]
        first += 1


def _insertion_sort(a, first, last):
    if first == last:
        return
    for i in range(first + 1, last):
        if _lt(a[i], a[first]):
            val = a[i]
            a[first + 1:i + 1] = a[first:i]
            a[first] = val
        else:
            val = a[i]
            j = i
            while _lt(val, a[j - 1]):
                a[j] = a[j - 1]
                j -= 1
            a[j] = val


def _push_heap(a, first, hole, top, value):
    parent = (hole - 1) // 2
    while hole > top and _lt(a[first + parent], value):
        a[first + hole] = a[first + parent]
        hole = parent
        parent = (hole - 1) // 2
    a[first + hole] = value


def _adjust_heap(a, first, hole, length, value):
    top = hole
    child = hole
    while child < (length - 1) // 2:
        child = 2 * (child + 1)
        if _lt(a[first + child], a[first + child - 1]):
            child -= 1
        a[first + hole] = a[first + child]
        hole = child
    if (length & 1) == 0 and child == (length - 2) // 2:
        child = 2 * (child + 1)
        a[first + hole] = a[first + child - 1]
        hole = child - 1
    _push_heap(a, first, hole, top, value)


def _make_heap(a, first, last):
    length = last - first
    if length < 2:
        return
    parent = (length - 2) // 2
    while True:
        _adjust_heap(a, first, parent, length, a[first + parent])
        if parent == 0:
            return
        parent -= 1


def _heap_select(a, first, middle, last):
    _make_heap(a, first, middle)
    for i in range(middle, last):
        if _lt(a[i], a[first]):
            value = a[i]
            a[i] = a[first]
            _adjust_heap(a, first, 0, middle - first, value)


def nth_element(a, nth):
    first, last = 0, len(a)
    if first == last or nth == last:
        return
    depth = 2 * ((last - first).bit_length() - 1)
    while last - first > 3:
        if depth == 0:
            _heap_select(a, first, nth + 1, last)
            a[first], a[nth] = a[nth], a[first]
            return
        depth -= 1
        mid = first + (last - first) // 2
        _move_median_to_first(a, first, first + 1, mid, last - 1)
        cut = _unguarded_partition(a, first + 1, last, first)
        if cut <= nth:
            first = cut
        else:
            last = cut
    _insertion_sort(a, first, last)


def topk_smallest_set(values, k):
    """Index set torch.topk(values, k, largest=False) returns on CPU (k*64 > n)."""
    n = len(values)
    if k > n:
        raise RuntimeError("selected index k out of range")
    q = [(float(values[j]), j) for j in range(n)]
    nth_element(q, k - 1)
    return sorted(j for _, j in q[:k])


# ---------------------------------------------------------------------------
# The same selection as the device computes it: one element per lane of a G-lane group
# (csrc/swarm_dl.h knn_tie_rows_wave).  Each partition round of the introselect loop is one
# parallel step over the left stoppers L_1 < L_2 < ... (!(v < pivot) in [first+1, last)) and the
# right stoppers R_1 > R_2 > ... (!(pivot < v) in [first, last)): the scans swap (L_t, R_t)
# exactly for t <= T, T = #{t : L_t < R_t}, and return L_1 (T = 0) or min(L_{T+1}, R_T).
# Readable restatement for the tests; pinned to torch.topk by tests/test_cpu_host.py.

def _sel_low(m, t):
    for _ in range(t - 1):
        m &= m - 1
    return (m & -m).bit_length() - 1


def _sel_high(m, t):
    for _ in range(t - 1):
        m &= ~(1 << (m.bit_length() - 1))
    return m.bit_length() - 1


def nth_element_lanes(a, nth):
    """nth_element on a list of (value, index) pairs, lane-parallel form (see above)."""
    n = len(a)
    first, last = 0, n
    if first == last or nth == last:
        return
    depth = 2 * (n.bit_length() - 1)
    while last - first > 3:
        if depth == 0:   # depth limit: the serial heap_select (as kv_nth_element)
            _heap_select(a, first, nth + 1, last)
            a[first], a[nth] = a[nth], a[first]
            return
        depth -= 1
        mid = first + (last - first) // 2
        x, y, z = first + 1, mid, last - 1
        if _lt(a[x], a[y]):
            pick = y if _lt(a[y], a[z]) else (z if _lt(a[x], a[z]) else x)
        elif _lt(a[x], a[z]):
            pick = x
        else:
            pick = z if _lt(a[y], a[z]) else y
        a[first], a[pick] = a[pick], a[first]
        pv = a[first]
        lm = sum(1 << e for e in range(first + 1, last) if not _lt(a[e], pv))
        rm = sum(1 << e for e in range(first, last) if not _lt(pv, a[e]))
        T = sum(1 for e in range(n) if lm >> e & 1 and bin(rm >> (e + 1)).count("1") >= bin(lm & ((1 << e) - 1)).count("1") + 1)
        src = list(range(n))
        for e in range(n):
            if lm >> e & 1:
                t = bin(lm & ((1 << e) - 1)).count("1") + 1
                if t <= T:
                    src[e] = _sel_high(rm, t)
            if rm >> e & 1:
                s = bin(rm >> (e + 1)).count("1") + 1
                if s <= T:
                    src[e] = _sel_low(lm, s)
        a[:] = [a[s] for s in src]
        cut = _sel_low(lm, 1)
        if T > 0:
            cut = _sel_high(rm, T)
            if bin(lm).count("1") > T:
                cut = min(cut, _sel_low(lm, T + 1))
        if cut <= nth:
            first = cut
        else:
            last = cut
    # insertion sort of <= 3 elements == stable sort by value
    a[first:last] = sorted(a[first:last], key=lambda kv: kv[0])


def topk_smallest_set_lanes(values, k):
    """topk_smallest_set through the lane-parallel restatement."""
    n = len(values)
    if k > n:
        raise RuntimeError("selected index k out of range")
    q = [(float(values[j]), j) for j in range(n)]
    nth_element_lanes(q, k - 1)
    return sorted(j for _, j in q[:k])


def topk_smallest_set_slots(values, k):
    """The round-3 device form (csrc/swarm_dl.h knn_tie_rows_wave): the same rounds as
    nth_element_lanes, with the swap partners found through rank slots (each left stopper
    publishes its index at its rank in an L row, each right stopper in an R row; a pair's
    members read each other) and the cut read from those rows; the closing insertion sort is
    replaced by its set: [0, first) plus the range elements of stable rank <= nth - first."""
    n = len(values)
    if k > n:
        raise RuntimeError("selected index k out of range")
    a = [(float(values[j]), j) for j in range(n)]
    nth = k - 1
    first, last = 0, n
    depth = 2 * (n.bit_length() - 1)
    heap = False
    while last - first > 3:
        if depth == 0:
            heap = True
            break
        depth -= 1
        mid = first + (last - first) // 2
        x, y, z = first + 1, mid, last - 1
        vx, vy, vz = a[x][0], a[y][0], a[z][0]
        xy, yz, xz = vx < vy, vy < vz, vx < vz
        py = (xy and yz) or (not xy and not xz and not yz)
        pz = (xy and not yz and xz) or (not xy and not xz and yz)
        pick = y if py else (z if pz else x)
        a[first], a[pick] = a[pick], a[first]
        pv = a[first][0]
        L = [e for e in range(first + 1, last) if not a[e][0] < pv]            # ascending
        R = [e for e in reversed(range(first, last)) if not pv < a[e][0]]      # descending
        T = sum(1 for t in range(min(len(L), len(R))) if L[t] < R[t])
        src = list(range(n))
        for t in range(T):                 # a lane that is R_t wins over being L_t', as on the device
            src[L[t]] = R[t]
        for t in range(T):
            src[R[t]] = L[t]
        a = [a[s] for s in src]
        cut = L[0] if T == 0 else (min(R[T - 1], L[T]) if len(L) > T else R[T - 1])
        if cut <= nth:
            first = cut
        else:
            last = cut
    if heap:
        _heap_select(a, first, nth + 1, last)
        a[first], a[nth] = a[nth], a[first]
        return sorted(j for _, j in a[:k])
    sel = list(range(first))
    for e in range(first, last):
        rank = sum(1 for j in range(first, last) if a[j][0] < a[e][0] or (a[j][0] == a[e][0] and j < e))
        if rank <= nth - first:
            sel.append(e)
    return sorted(a[e][1] for e in sel)


def rank_signature(values):
    """The tie memo's key (csrc/swarm_dl.h knn_masks_wave): lt_j = #{l : d_l < d_j} per
    element.  d_a < d_b iff lt_a < lt_b and d_a == d_b iff lt_a == lt_b, so the signature fixes
    every comparison introselect makes and with it the selected set."""
    return tuple(sum(1 for w in values if w < v) for v in values)


# A boundary-tie row (n = 15, k = 9: two 9s straddle the k-th place) whose introselect runs out
# of depth and ends in heap_select (found by search; exercised on the GPU by
# tests/test_gpu_parity.py test_acting_knn_ties_match_torch_topk)
HEAP_PATH_ROW = ([1, 12, 4, 11, 5, 13, 10, 14, 9, 8, 2, 3, 0, 6, 9], 9)
