// swarm_peer.hip — the peer exchange's setup calls (uncached exchange buffers, HIP IPC) and the
// standalone peer all-reduce.  The fused variant lives in swarm_td.hip (grad_reduce_kernel<1>).
// The reference has no distributed code (SURVEY.md §2 "Parallelism / comm backend: absent"); the
// collective this replaces is the build's own RCCL all_reduce(grad) (dist.py allreduce_grad_).
#include "swarm_peer.h"

namespace swarm {

// 16 columns x 8 source ranks per block (region 1 of the exchange buffer)
constexpr int kPeerArCols = 16;
__global__ __launch_bounds__(kPeerArCols * SWARM_PEER_MAX) void peer_allreduce_kernel(swarm_peer P, float* x, int n) {
  __shared__ float mine[kPeerArCols];
  __shared__ float rv[SWARM_PEER_MAX][kPeerArCols];
  const int c = threadIdx.x % kPeerArCols, q = threadIdx.x / kPeerArCols;
  const int col = blockIdx.x * kPeerArCols + c;
  if (q == 0) mine[c] = col < n ? x[col] : 0.0f;
  __syncthreads();
  peer_exchange<kPeerArCols>(P, 1, blockIdx.x, q, c, col, n, mine, rv);
  if (q == 0 && col < n) {
    float tot = rv[0][c];
    for (int w = 1; w < P.world_size; ++w) tot = tot + rv[w][c];
    x[col] = tot;
  }
}

}  // namespace swarm

using namespace swarm;

static_assert(sizeof(hipIpcMemHandle_t) == SWARM_PEER_HANDLE_BYTES, "IPC handle size");
static_assert((N_PARAMS + 1 + kPeerArCols - 1) / kPeerArCols <= kPeerSeqRegion, "peer seq region");

extern "C" {

int64_t swarm_peer_buffer_bytes(void) { return (int64_t)(peer_granules() * sizeof(unsigned long long)); }

int swarm_peer_alloc(void** buf) {
  if (!buf) return SWARM_E_BADARG;
  *buf = nullptr;
  void* p = nullptr;
  const size_t bytes = peer_granules() * sizeof(unsigned long long);
  // uncached: a peer's xGMI stores land in this GPU's HBM, and this GPU's polling loads must
  // not be served by a stale L2 line
  hipError_t e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(p, 0, bytes);   // tag 0 is never published
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    (void)hipFree(p);
    return (int)e;
  }
  *buf = p;
  return 0;
}

int swarm_peer_free(void* buf) { return buf ? (int)hipFree(buf) : 0; }

int swarm_peer_ipc_handle(void* buf, void* handle) {
  if (!buf || !handle) return SWARM_E_BADARG;
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, buf);
  if (e != hipSuccess) return (int)e;
  __builtin_memcpy(handle, &h, sizeof(h));
  return 0;
}

int swarm_peer_ipc_open(const void* handle, void** buf) {
  if (!handle || !buf) return SWARM_E_BADARG;
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  *buf = nullptr;
  return (int)hipIpcOpenMemHandle(buf, h, hipIpcMemLazyEnablePeerAccess);
}

int swarm_peer_ipc_close(void* buf) { return buf ? (int)hipIpcCloseMemHandle(buf) : 0; }

int swarm_peer_allreduce(const swarm_peer* peer, float* x, int32_t n, void* stream) {
  if (int e = check_peer(peer)) return e;
  if (!x || n < 1 || n > N_PARAMS + 1) return SWARM_E_BADARG;
  hipLaunchKernelGGL(peer_allreduce_kernel, dim3((n + kPeerArCols - 1) / kPeerArCols), dim3(kPeerArCols * SWARM_PEER_MAX),
                     0, (hipStream_t)stream, *peer, x, n);
  return (int)hipGetLastError();
}

}  // extern "C"
