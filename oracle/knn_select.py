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
