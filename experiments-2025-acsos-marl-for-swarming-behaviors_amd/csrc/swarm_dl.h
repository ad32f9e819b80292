// swarm_dl.h — GCN.forward of one graph per wave entirely in the MFMA 16x16x4 f32
// accumulator layout ("D layout", swarm_wpg.h): lane l -> column c = l & 15 (a node
// slot: node n = 16 ct + c of column tile ct) and row group p = l >> 4; register
// (t, r) of a 32-wide per-node vector is hidden feature 16 t + 4 p + r.
//
// Every dense product is an MFMA whose B operand is the previous stage's registers:
//   conv1.lin   H^T = W X^T            (K = 7 -> 2 k-steps; X straight from the state)
//   aggregate   O^T = H^T C^T          (K = NS source slots; C = attention coefficients)
//   lin1        Z^T = W1 tanh(O)^T     (K = 32; k-step (t, r) <-> feature 16 t + 4 p + r)
//   lin2        Q^T = W2 relu(Z)^T
// Per-node scalars (attention scores) are partial dot products reduced over the four
// row groups with permlane swaps; node-to-node data (scores, positions, the H rows the
// aggregation reads, Q rows) goes through wave-private LDS with wave-scope syncs.
//
// GCN.forward: src/training/train_gcn_dqn.py:59-70 (GATConv -> tanh -> lin1 -> relu
// -> lin2); GATConv math: PyG 2.5.3 (heads 1, add_self_loops False).
#pragma once
#include "swarm_wpg.h"

namespace swarm {

// sum over the four row groups (lanes l, l^16, l^32, l^48), bitwise identical in all four
__device__ inline float row4_sum(float x) {
  const int xi = __float_as_int(x);
  const auto a = __builtin_amdgcn_permlane16_swap(xi, xi, false, false);
  const float y = __int_as_float((int)a[0]) + __int_as_float((int)a[1]);
  const int yi = __float_as_int(y);
  const auto b = __builtin_amdgcn_permlane32_swap(yi, yi, false, false);
  return __int_as_float((int)b[0]) + __int_as_float((int)b[1]);
}

// pick v[4 k + p] for this lane's row group p (register arrays cannot be indexed by lane)
template <int M>
__device__ inline float pick4(const float (&v)[M], int k, int p) {
  const float a = v[4 * k], b = v[4 * k + 1], c = v[4 * k + 2], d = v[4 * k + 3];
  return p == 0 ? a : (p == 1 ? b : (p == 2 ? c : d));
}

template <int NS>
struct DGeom {
  static constexpr int CT = (NS + 15) / 16;   // column tiles of 16 node slots
  int lane, c, p;
  int gid;      // env (acting) or batch index (TD) of this wave; 0 if idle
  bool live;
};

template <int NS>
__device__ inline DGeom<NS> make_dgeom(int wave_gid, int count) {
  DGeom<NS> d;
  d.lane = threadIdx.x & 63;
  d.c = d.lane & 15;
  d.p = d.lane >> 4;
  d.live = wave_gid < count;
  d.gid = d.live ? wave_gid : 0;
  return d;
}

// per-lane forward state; index ct = column tile (node n = 16 ct + c)
template <int NS>
struct DFwd {
  static constexpr int CT = DGeom<NS>::CT;
  float x[CT][2];            // X[n][p], X[n][4 + p] (features: px py vx vy gx gy id 0)
  float t[CT][2][4];         // tanh(conv out)
  float zr[CT][2][4];        // relu(lin1)
  float cf[CT][NS];          // attention coefficient of the in-edge u -> n (0 if none)
  float sdst[CT];            // destination score of n
  float q[CT][kActions];     // Q row of n
};

// features of node n for this lane's two k-slots (p, 4 + p) from its state (pos, vel)
__device__ inline void node_x(float px, float py, float vx, float vy, int agent, int p, float x[2]) {
  x[0] = p == 0 ? px : (p == 1 ? py : (p == 2 ? vx : vy));
  x[1] = p == 0 ? kGoalX : (p == 1 ? kGoalY : (p == 2 ? (float)agent : 0.0f));
}

// multiplicity m(u -> n) (complete: train_gcn_dqn.py:101-108; kNN: simulator.py:15-24;
// dense: caller-supplied [B][N][N]).  A wave holds NS / GS graphs of GS slots each;
// slots of different graphs are never connected.
template <int NS, int GS = NS>
__device__ inline int in_mult(int u, int n, int N, int graph, const WSmall<NS>& sm, const uint8_t* __restrict__ dense,
                              int gid) {
  if constexpr (GS < NS) {
    if (u / GS != n / GS) return 0;
  }
  const int ju = (GS < NS) ? u % GS : u, jn = (GS < NS) ? n % GS : n;   // columns past NS: jn >= N
  if (ju >= N || jn >= N) return 0;
  if (graph == SWARM_GRAPH_COMPLETE) return (ju != jn ? 1 : 0) + ((ju == 0 && jn == 0) ? 1 : 0);
  if (graph == SWARM_GRAPH_KNN)
    return (int)((sm.knn[u] >> jn) & 1u) + (int)((sm.knn[n] >> ju) & 1u) + ((ju == 0 && jn == 0) ? 1 : 0);
  if (graph == SWARM_GRAPH_RADIUS)   // symmetric neighbour sets: one edge per ordered pair
    return (int)((sm.knn[n] >> ju) & 1u) + ((ju == 0 && jn == 0) ? 1 : 0);
  return (int)dense[((size_t)gid * N + ju) * N + jn];
}

// all in-edge multiplicities of target n, m[j] for source base + j (base = first slot of
// n's graph); the graph-type switch is taken once and each case is branch-free
template <int NS, int GS = NS>
__device__ inline void in_mults(int n, int N, int graph, const WSmall<NS>& sm, const uint8_t* __restrict__ dense,
                                int gid, int m[GS]) {
  const int jn = (GS < NS) ? n % GS : n;
  const int base = (GS < NS) ? (n / GS) * GS : 0;
  const bool tv = jn < N;
  if (graph == SWARM_GRAPH_COMPLETE) {
#pragma unroll
    for (int j = 0; j < GS; ++j) m[j] = (tv && j < N) ? (int)(j != jn) + (int)(j == 0 && jn == 0) : 0;
  } else if (graph == SWARM_GRAPH_KNN) {
    const uint32_t kn = sm.knn[min(n, NS - 1)];
#pragma unroll
    for (int j = 0; j < GS; ++j)
      m[j] = (tv && j < N) ? (int)((sm.knn[base + j] >> jn) & 1u) + (int)((kn >> j) & 1u) + (int)(j == 0 && jn == 0) : 0;
  } else if (graph == SWARM_GRAPH_RADIUS) {
    const uint32_t kn = sm.knn[min(n, NS - 1)];
#pragma unroll
    for (int j = 0; j < GS; ++j) m[j] = (tv && j < N) ? (int)((kn >> j) & 1u) + (int)(j == 0 && jn == 0) : 0;
  } else {
#pragma unroll
    for (int j = 0; j < GS; ++j) m[j] = (tv && j < N) ? (int)dense[((size_t)gid * N + j) * N + jn] : 0;
  }
}

// radius-neighbour row of slot n over its graph: bit j = local node j != n with
// |p_j - p_n| <= r (the kNN build's fp32 distance expression, simulator.py:18)
template <int NS, int GS = NS>
__device__ inline uint32_t radius_mask_node(int n, int N, float r, const WSmall<NS>& sm) {
  const int base = (GS < NS) ? (n / GS) * GS : 0;
  const int jn = (GS < NS) ? n % GS : n;
  if (jn >= N) return 0u;
  const float xi = sm.px[n], yi = sm.py[n];
  uint32_t m = 0u;
#pragma unroll
  for (int j = 0; j < GS; ++j) {
    const float d = norm2(sm.px[base + j] - xi, sm.py[base + j] - yi);
    m |= (j < N && j != jn && d <= r) ? (1u << j) : 0u;
  }
  return m;
}

// kNN row of slot n over its graph (positions in sm; bit j = local node j).  q: GS
// entries of lane-private LDS for the boundary-tie path.
template <int NS, int GS = NS>
__device__ inline uint32_t knn_mask_node(int n, int N, int k, const WSmall<NS>& sm, KV* q) {
  float d[GS];
  const int base = (GS < NS) ? (n / GS) * GS : 0;
  const float xi = sm.px[n], yi = sm.py[n];
#pragma unroll
  for (int j = 0; j < GS; ++j) d[j] = (j < N) ? norm2(sm.px[base + j] - xi, sm.py[base + j] - yi) : 0.0f;
  return topk_smallest_mask<GS>(d, N, k, q);
}

static __device__ inline void kv_heap_select_swap(KV* a, int first, int nth, int last) {
  kv_heap_select(a, first, nth + 1, last);
  kv_swap(a, first, nth);
}

// The boundary-tie rows of knn_masks_wave, G lanes per row (one element per lane, G >= the
// graph's node count): libstdc++'s introselect (swarm_knn.h kv_nth_element) restated on the
// group's lanes.  Median-of-3 is a swap of two lanes; the unguarded partition is one step:
// with L_1 < L_2 < ... the left stoppers (!(v < pivot), from first + 1) and R_1 > R_2 > ...
// the right stoppers (!(pivot < v), down to the pivot itself), the scans swap (L_t, R_t)
// exactly while L_t < R_t (t <= T) and return cut = L_1 (T = 0) or min(L_{T+1}, R_T) — every
// scan between two swaps runs over unswapped elements, and each swapped element is a stopper
// for the other scan.  The final insertion sort of <= 3 elements is a stable rank sort.  The
// heap_select branch (depth limit) runs serially in LDS as before.  Checked against
// torch.topk on 60,000 tie-heavy rows (n 4..16) before it went in; the GPU tests compare the
// sets with torch.topk (oracle knn_sets) and the recorded reference actions.
// tb: ballot with bit n * lpn set for every tie row n; q: GS KV entries of LDS per slot.
// Every per-group decision is a select instead of a branch.  Rows whose count test fails in a
// formation that persists (stacked agents keep a boundary tie every tick) run this every tick
// at one wave per SIMD,
// where a wave issues one instruction per 4 cycles: its instruction count is the acting
// launch's tail, hence the shape of a round:
//  - one hop of four values (the one at `first` and the three median candidates); the median
//    swap is applied locally (v1) and composed into the partition's gather;
//  - the partition's swap pairs (L_t, R_t), t <= T, meet through LDS: each left stopper
//    publishes its lane at slot rank - 1 of the group's L row, each right stopper at its rank
//    of the R row, and a lane of a pair reads its partner's lane; the cut (L_1, or the smaller
//    of R_T and L_(T+1)) is read from the same rows;
//  - one hop of (value, id).
// The rows' rounds run in lockstep; a group whose range is done keeps its lanes until the
// wave's last group finishes.  The finish needs no data movement: the selected set is every id
// left of `first` plus the range's elements whose stable rank (kv_insertion_sort's order) is
// at most nth - first.  q: the wave's KV scratch, reused as the L / R rows (2 G ints per group).
template <int NS, int GS>
__device__ inline void knn_tie_rows_wave(int lane, int N, int k, unsigned long long tb, int lpn, WSmall<NS>& sm,
                                         const float* __restrict__ dn, KV* q) {
  constexpr int G = GS <= 8 ? 8 : 16;   // lanes per row
  constexpr int NG = 64 / G;
  static_assert(NG * 2 * G <= 2 * NS * GS, "L / R rows fit the KV scratch");
  const int g = lane / G, e = lane % G, gb = lane - e;
  const int gb4 = gb << 2;
  int* const lr = reinterpret_cast<int*>(q) + g * 2 * G;   // [0, G): L_t's lane at t - 1; [G, 2G): R_t's
  auto gballot = [&](bool x) -> uint32_t {
    return (uint32_t)((__builtin_amdgcn_ballot_w64(x) >> gb) & ((1ull << G) - 1ull));
  };
  auto any = [](bool x) -> bool { return __builtin_amdgcn_ballot_w64(x) != 0ull; };
  // lane `from` of the group (ds_bpermute takes the lane modulo 64: out-of-range indices of
  // finished groups read some lane and are discarded)
  auto hop = [&](float x, int from) -> float {
    return __int_as_float(__builtin_amdgcn_ds_bpermute((from << 2) + gb4, __float_as_int(x)));
  };
  auto hopi = [&](int x, int from) -> int { return __builtin_amdgcn_ds_bpermute((from << 2) + gb4, x); };
  const int nth = k - 1;
  const int depth0 = 2 * floor_log2(N);
  const uint32_t below = (1u << e) - 1u;
  while (tb) {   // wave-uniform: up to NG tie rows per pass, group g takes the g-th remaining row
    int bit = -1;
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const int b = tb ? __ffsll((long long)tb) - 1 : -1;
      bit = i == g ? b : bit;
      tb &= tb - 1ull;
    }
    const bool row = bit >= 0;
    const int n = row ? bit / lpn : 0;
    float v = (row && e < N) ? dn[n * GS + e] : 0.0f;
    int id = e;
    int first = 0, last = N, depth = depth0;
    bool heap = false;
    while (true) {   // wave-uniform trip count: the longest row's rounds
      const bool open = row && !heap && last - first > 3;
      heap = heap || (open && depth == 0);
      const bool live = open && depth > 0;
      if (!any(live)) break;
      const int mid = first + (last - first) / 2;
      const float v0 = hop(v, first), vx = hop(v, first + 1), vy = hop(v, mid), vz = hop(v, last - 1);
      // kv_move_median_to_first(first, first + 1, mid, last - 1), as masks (no short circuits:
      // the compiler keeps selects where nested conditionals become branches)
      const bool xy = vx < vy, yz = vy < vz, xz = vx < vz;
      const bool py = (xy && yz) || (!xy && !xz && !yz);
      const bool pz = (xy && !yz && xz) || (!xy && !xz && yz);
      const int pick = py ? mid : (pz ? last - 1 : first + 1);
      const float pv = py ? vy : (pz ? vz : vx);   // the pivot, now at `first`
      const float v1 = e == first ? pv : (e == pick ? v0 : v);
      const bool in = live && e >= first && e < last;
      const bool is_l = in && e != first && !(v1 < pv);   // left stopper (scan from first + 1)
      const bool is_r = in && !(pv < v1);                 // right stopper (scan down to the pivot)
      const uint32_t lm = gballot(is_l), rm = gballot(is_r);
      const int tl = __popc(lm & below) + 1;      // rank among the left stoppers, ascending
      const int above = __popc(rm >> (e + 1));    // right stoppers after e
      const int tr = above + 1;                   // a right stopper's rank, descending
      wave_lds_sync();                            // the previous round's reads are done
      if (is_l) lr[tl - 1] = e;
      if (is_r) lr[G + tr - 1] = e;
      const int T = __popc(gballot(is_l && above >= tl));   // pairs with L_t < R_t
      wave_lds_sync();
      const bool take_r = is_r && tr <= T, take_l = is_l && tl <= T;
      const int partner = lr[take_r ? tr - 1 : G + tl - 1];   // R_t reads L_t, L_t reads R_t
      const int cut_r = lr[G + max(T, 1) - 1], cut_l = lr[min(T, G - 1)];
      int src = (take_r || take_l) ? partner : e;
      src = src == first ? pick : (src == pick ? first : src);   // through the median swap
      src = live ? src : e;
      v = hop(v, src);
      id = hopi(id, src);
      const int cut = T > 0 ? (__popc(lm) > T ? min(cut_r, cut_l) : cut_r) : __ffs(lm) - 1;
      first = (live && cut <= nth) ? cut : first;
      last = (live && cut > nth) ? cut : last;
      depth -= live ? 1 : 0;
    }
    bool sel = e < k;   // heap rows: heap_select + swap leaves the set in [0, k)
    if (any(heap)) {   // depth limit: heap_select + swap, serially (kv_nth_element)
      KV* a = q + n * GS;
      wave_lds_sync();
      if (heap && e < N) a[e] = KV{v, id};
      wave_lds_sync();
      if (heap && e == 0) kv_heap_select_swap(a, first, nth, last);
      wave_lds_sync();
      if (heap && e < N) { v = a[e].v; id = a[e].i; }
    }
    {   // kv_insertion_sort of [first, last) (<= 3 elements) is stable: the range's element of
        // stable rank r lands at first + r, so it is selected iff r <= nth - first
      const bool in = e >= first && e < last;
      int rank = 0;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int pj = first + j;
        const float vj = hop(v, pj);
        rank += (pj < last && (vj < v || (vj == v && pj < e))) ? 1 : 0;
      }
      sel = heap ? sel : (e < first || (in && rank <= nth - first));
    }
    // OR of the group's selected ids by DPP inside the 16-lane row: quad xor 1, quad xor 2,
    // half-row mirror (i <-> 7 - i), and for 16-lane groups the row mirror
    uint32_t mm = sel ? (1u << id) : 0u;
    mm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mm, 0xB1, 0xF, 0xF, false);
    mm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mm, 0x4E, 0xF, 0xF, false);
    mm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mm, 0x141, 0xF, 0xF, false);
    if (G == 16) mm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mm, 0x140, 0xF, 0xF, false);
    if (row && e == 0) sm.knn[n] = mm;
    wave_lds_sync();   // the next pass rewrites q
  }
}

// kNN rows of every slot of the wave at once (NS <= 16): lane l serves slot n = l / LPN and
// the candidates j = l % LPN + LPN i of n's graph.  Each pair distance is computed once
// (the same fp32 expression as knn_mask_node), the graph's distance rows meet in LDS
// (dn), and the set {j : #{l : d_l < d_j} < k} is assembled from wave ballots.  Slots
// whose count test fails (a boundary tie) run the introselect restatement knn_tie_rows_wave
// with its work space in LDS (q).  Writes sm.knn[n].
// memo (acting waves; nullptr elsewhere): the last tie row's result per slot, keyed by the
// row's rank signature: 4 bits of lt_j = #{l : d_l < d_j} per candidate.  d_a < d_b exactly
// when lt_a < lt_b, and d_a == d_b exactly when lt_a == lt_b, so the signature fixes every
// comparison introselect makes, hence its permutation and the selected ids: a tie row whose
// signature equals the slot's memo takes the memo's set without running the tie path.  Stacked
// agents keep a boundary tie on every tick while their distance ORDER changes rarely, and such
// a slot otherwise re-runs the tie path every tick (the acting launch's tail).
template <int NS, int GS>
__device__ inline void knn_masks_wave(int lane, int N, int k, WSmall<NS>& sm, float* __restrict__ dn, KV* q,
                                      TieMemo<NS>* memo = nullptr) {
  constexpr int LPN = 64 / NS;          // lanes per slot
  constexpr int CPL = GS / LPN;         // candidates per lane
  static_assert(CPL >= 1 && GS % LPN == 0, "knn_masks_wave geometry");
  static_assert(GS <= 16, "4-bit ranks of at most 16 candidates in the 64-bit signature");
  const int n = lane / LPN, r = lane % LPN;
  const int base = (GS < NS) ? (n / GS) * GS : 0;
  const int jn = (GS < NS) ? n % GS : n;
  const bool nvalid = jn < N;
  const float xi = sm.px[n], yi = sm.py[n];
  float dv[CPL];
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int j = r + LPN * i;
    dv[i] = (j < N) ? norm2(sm.px[base + j] - xi, sm.py[base + j] - yi) : 0.0f;
    dn[n * GS + j] = dv[i];
  }
  wave_lds_sync();
  float row[GS];
  lds_load<GS>(dn + n * GS, row);
  uint32_t mask = 0;
  uint32_t sig_lo = 0, sig_hi = 0;   // this lane's candidates' 4-bit ranks
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int j = r + LPN * i;
    int lt = 0;
#pragma unroll
    for (int l = 0; l < GS; ++l) lt += (l < N && row[l] < dv[i]) ? 1 : 0;
    const uint64_t b = __ballot(nvalid && j < N && lt < k);
    mask |= (uint32_t)((b >> (n * LPN)) & ((1ull << LPN) - 1ull)) << (LPN * i);
    const uint32_t nib = j < N ? (uint32_t)lt : 0u;
    if (LPN * i < 8) sig_lo |= nib << (4 * j);   // all of this i's candidates are below 8
    else sig_hi |= nib << (4 * (j - 8));
  }
  const bool tie = r == 0 && nvalid && __popc(mask) != k;
  bool hit = false;
  uint32_t hit_mask = 0u;
  if (memo) {
    // OR the slot's LPN lanes (aligned groups inside a 16-lane row): quad xor 1, quad xor 2,
    // and for 8-lane slots the half-row mirror
    sig_lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sig_lo, 0xB1, 0xF, 0xF, false);
    sig_hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sig_hi, 0xB1, 0xF, 0xF, false);
    if (LPN >= 4) {
      sig_lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sig_lo, 0x4E, 0xF, 0xF, false);
      sig_hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sig_hi, 0x4E, 0xF, 0xF, false);
    }
    if (LPN >= 8) {
      sig_lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sig_lo, 0x141, 0xF, 0xF, false);
      sig_hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sig_hi, 0x141, 0xF, 0xF, false);
    }
    static_assert(LPN == 4 || LPN == 8, "memo signature reduction covers 4- and 8-lane slots");
    if (tie) {
      hit = memo->sig_lo[n] == sig_lo && memo->sig_hi[n] == sig_hi;
      hit_mask = memo->mask[n];
    }
  }
  if (r == 0) sm.knn[n] = nvalid ? (hit ? hit_mask : mask) : 0u;
  const bool run = tie && !hit;
  const unsigned long long tb = __ballot(run);
  if (tb != 0ull) {
    // boundary ties: the introselect restatement, G lanes per row
#if SWARM_STAMPS == 1   // stamps build: per-wave tie-path entries (slot 27) and s_memtime cycles in it (slot 28)
    const long long s0 = clock64();
#endif
    wave_lds_sync();
    knn_tie_rows_wave<NS, GS>(lane, N, k, tb, LPN, sm, dn, q);
    wave_lds_sync();
    if (memo && run) {
      memo->sig_lo[n] = sig_lo;
      memo->sig_hi[n] = sig_hi;
      memo->mask[n] = sm.knn[n];
    }
#if SWARM_STAMPS == 1
    wave_lds_sync();
    const long long s1 = clock64();
    if (g_swarm_stamps && lane == 0) {
      unsigned long long* ws = g_swarm_stamps + ((size_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 32;
      ws[27] += 1ull;
      ws[28] += (unsigned long long)(s1 - s0);
      if ((unsigned long long)(s1 - s0) > ws[26]) ws[26] = (unsigned long long)(s1 - s0);
    }
#endif
  }
#if SWARM_STAMPS == 1
  if (memo && g_swarm_stamps && lane == 0 && __ballot(hit) != 0ull)   // slot 18: memo hits
    g_swarm_stamps[((size_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 32 + 18] += 1ull;
#endif
}

// Full GCN.forward.  F.x must hold the lane's features (zero for nodes >= N).  P is the
// padded LDS weight image.  Writes the H rows (and T / R rows if keep_tr) of V, the
// per-node scalars of V.sm, and leaves F.t / F.zr / F.cf / F.q for the backward.
template <int NS, int SB = -1, int GS = NS>
__device__ inline void dl_forward(const float* __restrict__ P, const DGeom<NS>& d, int N, int graph, int k, float radius, int conv,
                                  const uint8_t* __restrict__ dense, const WView<NS>& V, bool keep_tr, DFwd<NS>& F) {
#define DF_STAMP(i) do { if (SB >= 0) SWARM_STAMP(SB + (i)); } while (0)
  constexpr int CT = DGeom<NS>::CT;
  WSmall<NS>& sm = *V.sm;
  const int c = d.c, p = d.p;
  // ---- conv1.lin on MFMA (K = 7 padded to 8): A[f][k] = W[f][k], B[k][n] = X[n][k]
  float h[CT][2][4];
  {
    float a0[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      a0[t][0] = P[L_W + (16 * t + c) * kFeat + p];
      // read unconditionally (p = 3 reads the next row's first weight, inside the image) and
      // masked after: no branch around a masked LDS read at the head of every forward
      a0[t][1] = P[L_W + (16 * t + c) * kFeat + 4 + p];
      asm volatile("" : "+v"(a0[t][1]));
      a0[t][1] = (4 + p < kFeat) ? a0[t][1] : 0.0f;
    }
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        acc = mfma16(a0[t][0], F.x[ct][0], acc);
        acc = mfma16(a0[t][1], F.x[ct][1], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) h[ct][t][r] = acc[r];
      }
  }
  // ---- attention scores (h * att).sum(-1): 8 features per lane, then the 4 row groups
  float ssrc[CT];
  {
    const float4 s0 = *reinterpret_cast<const float4*>(P + L_ATT_SRC + 4 * p);
    const float4 s1 = *reinterpret_cast<const float4*>(P + L_ATT_SRC + 16 + 4 * p);
    const float4 d0 = *reinterpret_cast<const float4*>(P + L_ATT_DST + 4 * p);
    const float4 d1 = *reinterpret_cast<const float4*>(P + L_ATT_DST + 16 + 4 * p);
    const float as[2][4] = {{s0.x, s0.y, s0.z, s0.w}, {s1.x, s1.y, s1.z, s1.w}};
    const float ad[2][4] = {{d0.x, d0.y, d0.z, d0.w}, {d1.x, d1.y, d1.z, d1.w}};
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      float ps = 0.0f, pd = 0.0f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) { ps = ps + h[ct][t][r] * as[t][r]; pd = pd + h[ct][t][r] * ad[t][r]; }
      ssrc[ct] = row4_sum(ps);
      F.sdst[ct] = row4_sum(pd);
    }
  }
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int n = 16 * ct + c;
    if (n < NS) {
      *reinterpret_cast<float4*>(&V.H[n][4 * p]) = make_float4(h[ct][0][0], h[ct][0][1], h[ct][0][2], h[ct][0][3]);
      *reinterpret_cast<float4*>(&V.H[n][16 + 4 * p]) = make_float4(h[ct][1][0], h[ct][1][1], h[ct][1][2], h[ct][1][3]);
      if (p == 0) { sm.ssrc[n] = ssrc[ct]; sm.sdst[n] = F.sdst[ct]; sm.px[n] = F.x[ct][0]; }
      if (p == 1) sm.py[n] = F.x[ct][0];
    }
  }
  wave_lds_sync();
  DF_STAMP(0);
  if (graph == SWARM_GRAPH_KNN) {
    // work space in the wave's T / R rows (free until the aggregation writes T)
    if constexpr (NS <= 16) {
      knn_masks_wave<NS, GS>(d.lane, N, k, sm, &V.T[0][0], reinterpret_cast<KV*>(&V.R[0][0]), V.memo);
    } else {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int n = 16 * ct + c;
        // node n's GS entries of T / R (contiguous: 2 NS kRow floats >= 2 NS GS)
        KV* q = reinterpret_cast<KV*>(&V.T[0][0]) + (n < NS ? n : 0) * GS;
        if (n < NS && p == 0) sm.knn[n] = (((GS < NS) ? n % GS : n) < N) ? knn_mask_node<NS, GS>(n, N, k, sm, q) : 0u;
      }
    }
    wave_lds_sync();
  } else if (graph == SWARM_GRAPH_RADIUS) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int n = 16 * ct + c;
      if (n < NS && p == 0) sm.knn[n] = radius_mask_node<NS, GS>(n, N, radius, sm);
    }
    wave_lds_sync();
  }
  // ---- in-edge coefficients of target n (every row group computes them; PyG softmax
  //      exp(e - max) / (sum + 1e-16) with duplicate edges counted by multiplicity)
  if (conv == SWARM_CONV_GAT) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int n = 16 * ct + c, base = (GS < NS) ? (n / GS) * GS : 0;
      float e[GS];
      int m[GS];
      in_mults<NS, GS>(n, N, graph, sm, dense, d.gid, m);
      // the max over present edges as a tree (max is exact: the serial order's value, three
      // dependent steps instead of GS)
      float mx[GS];
#pragma unroll
      for (int j = 0; j < GS; ++j) {
        e[j] = leaky(sm.ssrc[base + j] + F.sdst[ct]);
        mx[j] = m[j] > 0 ? e[j] : -INFINITY;
      }
#pragma unroll
      for (int w = GS / 2; w >= 1; w >>= 1)
#pragma unroll
        for (int j = 0; j < w; ++j) mx[j] = fmaxf(mx[j], mx[j + w]);
      const float emax = mx[0];
      float den = 0.0f;
#pragma unroll
      for (int j = 0; j < GS; ++j) {
        e[j] = m[j] > 0 ? __expf(e[j] - emax) : 0.0f;
        den = den + (float)m[j] * e[j];
      }
      den = den + 1e-16f;
      const float inv = 1.0f / den;
      float cl[GS];
#pragma unroll
      for (int j = 0; j < GS; ++j) cl[j] = (float)m[j] * (e[j] * inv);
#pragma unroll
      for (int u = 0; u < NS; ++u) F.cf[ct][u] = (GS == NS || u / GS == n / GS) ? cl[u % GS] : 0.0f;
    }
  } else {
    // GCNConv (a13, parity unpinned): self loops collapse to weight 1, symmetric deg^-1/2
    float dis[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int n = 16 * ct + c, base = (GS < NS) ? (n / GS) * GS : 0;
      float deg = 0.0f;
#pragma unroll
      for (int j = 0; j < GS; ++j)
        if (j < N) deg = deg + (base + j == n ? 1.0f : (float)in_mult<NS, GS>(base + j, n, N, graph, sm, dense, d.gid));
      const int jn = (GS < NS) ? n % GS : n;
      dis[ct] = (jn < N && deg > 0.0f) ? 1.0f / sqrtf(deg) : 0.0f;
      if (n < NS && p == 0) sm.aux[n] = dis[ct];
    }
    wave_lds_sync();
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int n = 16 * ct + c;
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        const bool same = (GS == NS) || (u / GS == n / GS);
        const float w = (u == n) ? 1.0f : (float)in_mult<NS, GS>(u, n, N, graph, sm, dense, d.gid);
        const int ju = (GS < NS) ? u % GS : u, jn = (GS < NS) ? n % GS : n;
        F.cf[ct][u] = (same && ju < N && jn < N) ? (sm.aux[u] * w) * dis[ct] : 0.0f;
      }
    }
  }
  DF_STAMP(1);
  // ---- aggregate on MFMA: O^T[f][n] = sum_u H[u][f] C[n][u], K = NS source slots
  {
    float ah[2][NS / 4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < NS / 4; ++ks) ah[t][ks] = V.H[4 * ks + p][16 * t + c];
    const float4 b0 = *reinterpret_cast<const float4*>(P + L_BIAS + 4 * p);
    const float4 b1 = *reinterpret_cast<const float4*>(P + L_BIAS + 16 + 4 * p);
    const float bias[2][4] = {{b0.x, b0.y, b0.z, b0.w}, {b1.x, b1.y, b1.z, b1.w}};
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NS / 4; ++ks) {
        const float b = pick4(F.cf[ct], ks, p);
        o0 = mfma16(ah[0][ks], b, o0);
        o1 = mfma16(ah[1][ks], b, o1);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        F.t[ct][0][r] = tanh_fast(o0[r] + bias[0][r]);
        F.t[ct][1][r] = tanh_fast(o1[r] + bias[1][r]);
      }
      const int n = 16 * ct + c;
      if (keep_tr && n < NS) {
        *reinterpret_cast<float4*>(&V.T[n][4 * p]) = make_float4(F.t[ct][0][0], F.t[ct][0][1], F.t[ct][0][2], F.t[ct][0][3]);
        *reinterpret_cast<float4*>(&V.T[n][16 + 4 * p]) = make_float4(F.t[ct][1][0], F.t[ct][1][1], F.t[ct][1][2], F.t[ct][1][3]);
      }
    }
  }
  DF_STAMP(2);
  // ---- lin1 + relu on MFMA: Z^T = W1 tanh^T, the tanh registers are the B operand
  {
    float a1[2][2][4];   // [out tile t2][k tile t][r] = W1[16 t2 + c][16 t + 4 p + r]
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const float4 w = *reinterpret_cast<const float4*>(P + L_W1 + (16 * t2 + c) * kWRow + 16 * t + 4 * p);
        a1[t2][t][0] = w.x; a1[t2][t][1] = w.y; a1[t2][t][2] = w.z; a1[t2][t][3] = w.w;
      }
    const float4 bb0 = *reinterpret_cast<const float4*>(P + L_B1 + 4 * p);
    const float4 bb1 = *reinterpret_cast<const float4*>(P + L_B1 + 16 + 4 * p);
    const float b1v[2][4] = {{bb0.x, bb0.y, bb0.z, bb0.w}, {bb1.x, bb1.y, bb1.z, bb1.w}};
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      // the two output tiles' chains interleaved (independent accumulators: 32-cycle issue
      // instead of the 40-cycle dependent latency per MFMA); each chain keeps its k order
      f32x4 z[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int t2 = 0; t2 < 2; ++t2) z[t2] = mfma16(a1[t2][t][r], F.t[ct][t][r], z[t2]);
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float u = z[t2][r] + b1v[t2][r];
          F.zr[ct][t2][r] = u > 0.0f ? u : 0.0f;
        }
      }
      const int n = 16 * ct + c;
      if (keep_tr && n < NS) {
        *reinterpret_cast<float4*>(&V.R[n][4 * p]) = make_float4(F.zr[ct][0][0], F.zr[ct][0][1], F.zr[ct][0][2], F.zr[ct][0][3]);
        *reinterpret_cast<float4*>(&V.R[n][16 + 4 * p]) = make_float4(F.zr[ct][1][0], F.zr[ct][1][1], F.zr[ct][1][2], F.zr[ct][1][3]);
      }
    }
  }
  DF_STAMP(3);
  // ---- lin2 on MFMA: Q^T = W2 relu^T (A rows >= 9 zero); Q rows exchanged through LDS
  {
    float a2[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
      if (c < kActions) w = *reinterpret_cast<const float4*>(P + L_W2 + c * kWRow + 16 * t + 4 * p);
      a2[t][0] = w.x; a2[t][1] = w.y; a2[t][2] = w.z; a2[t][3] = w.w;
    }
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      f32x4 qa = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) qa = mfma16(a2[t][r], F.zr[ct][t][r], qa);
      const int n = 16 * ct + c;
      if (n < NS && p < 3) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int a = 4 * p + r;
          if (a < kActions) sm.Q[n][a] = qa[r] + P[L_B2 + a];
        }
      }
    }
  }
  wave_lds_sync();
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int n = min(16 * ct + c, NS - 1);
    const float4 q0 = *reinterpret_cast<const float4*>(&sm.Q[n][0]);
    const float4 q1 = *reinterpret_cast<const float4*>(&sm.Q[n][4]);
    F.q[ct][0] = q0.x; F.q[ct][1] = q0.y; F.q[ct][2] = q0.z; F.q[ct][3] = q0.w;
    F.q[ct][4] = q1.x; F.q[ct][5] = q1.y; F.q[ct][6] = q1.z; F.q[ct][7] = q1.w;
    F.q[ct][8] = sm.Q[n][8];
  }
  DF_STAMP(4);
#undef DF_STAMP
}

}  // namespace swarm
