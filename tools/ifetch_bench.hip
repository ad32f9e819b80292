// Diagnostic (round 5): what straight-line code costs a launch whose instruction caches start
// cold.  The fused tick's PMC (profiles/r05_icache_counters.json) shows every SQC refetching the
// code it runs at every launch; this times hipGraph chains of one kernel that runs the same
// dependent VALU chain either fully unrolled (K instructions of code) or as a loop of 16 (a few
// lines of code), one wave per CU, and prints the per-launch period of each.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/ifetch_bench tools/ifetch_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int K>
__global__ void __launch_bounds__(64) unrolled(float* out, float a, float b) {
  float x = out[threadIdx.x];
#pragma unroll
  for (int i = 0; i < K; ++i) x = __builtin_fmaf(x, a, b);
  out[threadIdx.x] = x;
}

template <int K>
__global__ void __launch_bounds__(64) rolled(float* out, float a, float b) {
  float x = out[threadIdx.x];
#pragma nounroll
  for (int i = 0; i < K / 16; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) x = __builtin_fmaf(x, a, b);
  }
  out[threadIdx.x] = x;
}

template <typename F>
static float period_us(F launch, hipStream_t s, int reps) {
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < reps; ++i) launch();
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int t = 0; t < 5; ++t) {
    hipEventRecord(e0, s);
    hipGraphLaunch(ge, s);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  return 1000.0f * best / reps;
}

template <int K>
static void run(float* buf, hipStream_t s) {
  const int blocks = 256, reps = 200;
  const float pu = period_us([&] { unrolled<K><<<blocks, 64, 0, s>>>(buf, 0.999f, 0.001f); }, s, reps);
  const float pr = period_us([&] { rolled<K><<<blocks, 64, 0, s>>>(buf, 0.999f, 0.001f); }, s, reps);
  printf("{\"fma_chain\": %d, \"unrolled_code_bytes\": %d, \"unrolled_us\": %.3f, \"rolled_us\": %.3f, \"extra_us\": %.3f}\n",
         K, 8 * K, pu, pr, pu - pr);
}

int main() {
  float* buf;
  hipMalloc(&buf, 64 * sizeof(float));
  hipMemset(buf, 0, 64 * sizeof(float));
  hipStream_t s;
  hipStreamCreate(&s);
  run<256>(buf, s);
  run<1024>(buf, s);
  run<2048>(buf, s);
  run<4096>(buf, s);
  run<8192>(buf, s);
  hipFree(buf);
  return 0;
}
