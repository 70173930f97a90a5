// Micro-benchmark (tools only): launch/latency floors for the env-step shapes.
// Times graph-replayed launch sequences with hipEvents; run under
// `rocprofv3 --kernel-trace --stats` for per-kernel durations.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/launch_micro tools/launch_micro.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__global__ __launch_bounds__(64) void k_null64(int64_t* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = blockIdx.x;
}
__global__ __launch_bounds__(256) void k_null256(int64_t* out) {
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = blockIdx.x;
}
// one read of 64 B per env (lane-per-row words), one 8-B write
__global__ __launch_bounds__(64) void k_rw64(const uint64_t* rows, int64_t* out) {
  const int lane = threadIdx.x;
  uint64_t v = lane < 4 ? rows[blockIdx.x * 4 + lane] : 0;
  v = __ballot(v != 0);
  if (lane == 0) out[blockIdx.x] = (int64_t)v;
}
// obs-shaped store: 10 float4 per lane per env (10 KiB per env), 1 wave per env
__global__ __launch_bounds__(64) void k_store64(float4* obs) {
  float4* o = obs + (size_t)blockIdx.x * 640 + threadIdx.x;
  const float f = (float)(threadIdx.x & 1);
#pragma unroll
  for (int c = 0; c < 10; ++c) o[c * 64] = make_float4(f, 0.f, f, 0.f);
}
// same bytes, 4 envs per 256-thread workgroup
__global__ __launch_bounds__(256) void k_store256(float4* obs) {
  const int env = blockIdx.x * 4 + (threadIdx.x >> 6);
  float4* o = obs + (size_t)env * 640 + (threadIdx.x & 63);
  const float f = (float)(threadIdx.x & 1);
#pragma unroll
  for (int c = 0; c < 10; ++c) o[c * 64] = make_float4(f, 0.f, f, 0.f);
}

typedef void (*Launch)(hipStream_t, void*, void*, int);

static float time_graph(hipStream_t s, Launch fn, void* a, void* b, int n, int reps) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < reps; ++i) fn(s, a, b, n);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s));  // warm
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return ms * 1000.f / reps;
}

static void L_null64(hipStream_t s, void* a, void*, int n) { k_null64<<<n, 64, 0, s>>>((int64_t*)a); }
static void L_null256(hipStream_t s, void* a, void*, int n) { k_null256<<<n / 4, 256, 0, s>>>((int64_t*)a); }
static void L_rw64(hipStream_t s, void* a, void* b, int n) { k_rw64<<<n, 64, 0, s>>>((const uint64_t*)b, (int64_t*)a); }
static void L_store64(hipStream_t s, void* a, void* b, int n) { k_store64<<<n, 64, 0, s>>>((float4*)b); }
static void L_store256(hipStream_t s, void* a, void* b, int n) { k_store256<<<n / 4, 256, 0, s>>>((float4*)b); }

int main(int argc, char** argv) {
  const int reps = 200;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  void *a, *b;
  CK(hipMalloc(&a, 32768 * 8 * 4));
  CK(hipMalloc(&b, (size_t)32768 * 640 * 16));
  CK(hipMemset(b, 1, (size_t)32768 * 640 * 16));
  const int ns[] = {4096, 32768};
  for (int n : ns) {
    printf("n=%d\n", n);
    printf("  null 1 wave/WG        %7.2f us\n", time_graph(s, L_null64, a, b, n, reps));
    printf("  null 4 waves/WG       %7.2f us\n", time_graph(s, L_null256, a, b, n, reps));
    printf("  read64B+write8B/env   %7.2f us\n", time_graph(s, L_rw64, a, b, n, reps));
    const float t64 = time_graph(s, L_store64, a, b, n, reps);
    const float t256 = time_graph(s, L_store256, a, b, n, reps);
    const double mb = (double)n * 10240 / 1e6;
    printf("  store 10KiB/env 1w/WG %7.2f us  (%.0f GB/s)\n", t64, mb / t64 * 1e3);
    printf("  store 10KiB/env 4w/WG %7.2f us  (%.0f GB/s)\n", t256, mb / t256 * 1e3);
  }
  return 0;
}
