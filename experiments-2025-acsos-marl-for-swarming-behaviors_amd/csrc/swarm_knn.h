// swarm_knn.h — the neighbour set CPU torch.topk(dist, k, largest=False) returns
// (simulator.py:18-19), reproduced exactly, for host and device.
//
// torch TopKImpl (k*64 > n): queue[j] = (dist_j, j); std::nth_element(begin,
// begin+k-1, end, [](x,y){return x.first < y.first;}); keep queue[0..k).
// With ties at the k-boundary the surviving indices depend on libstdc++'s
// __introselect, restated below step by step (median-of-3 to first, unguarded
// partition, insertion sort below 4 elements, heap_select when the depth limit
// 2*floor(log2 n) runs out).  Fast path: when the k smallest values are unique
// at the boundary the set is {j : #{l : d_l < d_j} < k}, which any selection
// algorithm returns; the introselect emulation runs only on boundary ties.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace swarm {

struct KV { float v; int i; };
__host__ __device__ inline bool kv_lt(const KV& a, const KV& b) { return a.v < b.v; }
__host__ __device__ inline void kv_swap(KV* a, int x, int y) { KV t = a[x]; a[x] = a[y]; a[y] = t; }

__host__ __device__ inline void kv_push_heap(KV* a, int first, int hole, int top, KV value) {
  int parent = (hole - 1) / 2;
  while (hole > top && kv_lt(a[first + parent], value)) {
    a[first + hole] = a[first + parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  a[first + hole] = value;
}

__host__ __device__ inline void kv_adjust_heap(KV* a, int first, int hole, int len, KV value) {
  const int top = hole;
  int child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (kv_lt(a[first + child], a[first + child - 1])) child--;
    a[first + hole] = a[first + child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    a[first + hole] = a[first + child - 1];
    hole = child - 1;
  }
  kv_push_heap(a, first, hole, top, value);
}

__host__ __device__ inline void kv_heap_select(KV* a, int first, int middle, int last) {
  const int len = middle - first;
  if (len >= 2) {
    for (int parent = (len - 2) / 2;; --parent) {
      kv_adjust_heap(a, first, parent, len, a[first + parent]);
      if (parent == 0) break;
    }
  }
  for (int i = middle; i < last; ++i) {
    if (kv_lt(a[i], a[first])) {
      KV value = a[i];
      a[i] = a[first];
      kv_adjust_heap(a, first, 0, len, value);
    }
  }
}

__host__ __device__ inline void kv_move_median_to_first(KV* a, int result, int x, int y, int z) {
  if (kv_lt(a[x], a[y])) {
    if (kv_lt(a[y], a[z])) kv_swap(a, result, y);
    else if (kv_lt(a[x], a[z])) kv_swap(a, result, z);
    else kv_swap(a, result, x);
  } else if (kv_lt(a[x], a[z])) kv_swap(a, result, x);
  else if (kv_lt(a[y], a[z])) kv_swap(a, result, z);
  else kv_swap(a, result, y);
}

__host__ __device__ inline int kv_unguarded_partition(KV* a, int first, int last, int pivot) {
  while (true) {
    while (kv_lt(a[first], a[pivot])) ++first;
    --last;
    while (kv_lt(a[pivot], a[last])) --last;
    if (!(first < last)) return first;
    kv_swap(a, first, last);
    ++first;
  }
}

__host__ __device__ inline void kv_insertion_sort(KV* a, int first, int last) {
  if (first == last) return;
  for (int i = first + 1; i < last; ++i) {
    KV val = a[i];
    if (kv_lt(val, a[first])) {
      for (int j = i; j > first; --j) a[j] = a[j - 1];
      a[first] = val;
    } else {
      int j = i;
      while (kv_lt(val, a[j - 1])) { a[j] = a[j - 1]; --j; }
      a[j] = val;
    }
  }
}

__host__ __device__ inline int floor_log2(int n) { int l = 0; while (n > 1) { n >>= 1; ++l; } return l; }

// std::nth_element(a, a+nth, a+n) with the less-than-on-value comparator
__host__ __device__ inline void kv_nth_element(KV* a, int n, int nth) {
  int first = 0, last = n;
  if (first == last || nth == last) return;
  int depth = 2 * floor_log2(last - first);
  while (last - first > 3) {
    if (depth == 0) {
      kv_heap_select(a, first, nth + 1, last);
      kv_swap(a, first, nth);
      return;
    }
    --depth;
    const int mid = first + (last - first) / 2;
    kv_move_median_to_first(a, first, first + 1, mid, last - 1);
    const int cut = kv_unguarded_partition(a, first + 1, last, first);
    if (cut <= nth) first = cut; else last = cut;
  }
  kv_insertion_sort(a, first, last);
}

// selection bitmask over j < n (n <= 32) of torch.topk(d, k, largest=False) on CPU.
// q: NMAX entries of work space for the tie path; on the device the callers pass a
// lane-private slice of LDS (a private array with data-dependent indices lives in
// scratch memory, one HBM round trip per introselect step).
template <int NMAX>
__host__ __device__ inline uint32_t topk_smallest_mask(const float* d, int n, int k, KV* q) {
  uint32_t mask = 0;
  int count = 0;
#pragma unroll
  for (int j = 0; j < NMAX; ++j) {
    if (j < n) {
      int lt = 0;
#pragma unroll
      for (int l = 0; l < NMAX; ++l) lt += (l < n && d[l] < d[j]) ? 1 : 0;
      if (lt < k) { mask |= 1u << j; ++count; }
    }
  }
  if (count == k) return mask;
#pragma unroll
  for (int j = 0; j < NMAX; ++j)
    if (j < n) { q[j].v = d[j]; q[j].i = j; }
  kv_nth_element(q, n, k - 1);
  mask = 0;
  for (int j = 0; j < k; ++j) mask |= 1u << q[j].i;
  return mask;
}

// the boundary-tie path alone (callers that already know the count test failed)
template <int NMAX>
__host__ __device__ inline uint32_t topk_tie_mask(const float* d, int n, int k, KV* q) {
#pragma unroll
  for (int j = 0; j < NMAX; ++j)
    if (j < n) { q[j].v = d[j]; q[j].i = j; }
  kv_nth_element(q, n, k - 1);
  uint32_t mask = 0;
  for (int j = 0; j < k; ++j) mask |= 1u << q[j].i;
  return mask;
}

template <int NMAX>
__host__ __device__ inline uint32_t topk_smallest_mask(const float* d, int n, int k) {
  KV q[NMAX];
  return topk_smallest_mask<NMAX>(d, n, k, q);
}

}  // namespace swarm
