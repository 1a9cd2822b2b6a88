// What a launch boundary costs against an in-kernel grid barrier (MI355X, one process, one stream).
//
//  (a) a HIP graph of NK tiny kernels (G blocks x 256 threads, each block writes one float4 per
//      thread of a 64 KiB buffer and reads the previous kernel's): time per kernel node;
//  (b) ONE kernel of G co-resident blocks doing the same NK dependent phases separated by a grid
//      barrier (relaxed agent-scope ticket counter, never reset, each block polls until the
//      phase's last ticket is taken; phase data written through with agent-scope atomic stores
//      and drained with vmcnt(0) before the ticket, read with agent-scope atomic loads).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/barrier_probe csrc/bench/barrier_probe.hip
// Run:   barrier_probe [G=256] [NK=24]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

__global__ __launch_bounds__(256) void phase_kernel(const float* __restrict__ in, float* __restrict__ out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = in[(i * 7) % n] * 0.5f + 1.f;
}

// NK phases in one launch; ticket = the grid-barrier counter (zeroed once, only ever advanced)
__global__ __launch_bounds__(256) void fused_kernel(float* a, float* b, int n, int nk, unsigned* ticket) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const unsigned G = gridDim.x;
  float* src = a;
  float* dst = b;
  for (int k = 0; k < nk; ++k) {
    if (i < n) {
      const float v = __hip_atomic_load(src + (i * 7) % n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dst + i, v * 0.5f + 1.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (t / G + 1) * G;
      const unsigned long long t0 = wall_clock64();
      while (__hip_atomic_load(ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > 25000000ull) break;  // 0.25 s: never in a healthy run
      }
    }
    __syncthreads();
    float* t = src;
    src = dst;
    dst = t;
  }
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 256;
  const int NK = argc > 2 ? atoi(argv[2]) : 24;
  const int n = G * 256;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  if (G > cus) {
    fprintf(stderr, "G = %d > %d CUs: the fused kernel's blocks would not all be resident\n", G, cus);
    return 2;
  }
  float *a, *b;
  unsigned* ticket;
  CK(hipMalloc(&a, n * sizeof(float)));
  CK(hipMalloc(&b, n * sizeof(float)));
  CK(hipMalloc(&ticket, sizeof(unsigned)));
  CK(hipMemset(a, 0, n * sizeof(float)));
  CK(hipMemset(b, 0, n * sizeof(float)));
  CK(hipMemset(ticket, 0, sizeof(unsigned)));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  // (a) graph of NK kernels
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int k = 0; k < NK; ++k) hipLaunchKernelGGL(phase_kernel, dim3(G), dim3(256), 0, st, k % 2 ? b : a, k % 2 ? a : b, n);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  // (b) graph of one fused kernel
  hipGraph_t gf;
  hipGraphExec_t gfe;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(fused_kernel, dim3(G), dim3(256), 0, st, a, b, n, NK, ticket);
  CK(hipStreamEndCapture(st, &gf));
  CK(hipGraphInstantiate(&gfe, gf, nullptr, nullptr, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    for (int w = 0; w < 20; ++w) {
      CK(hipGraphLaunch(ge, st));
      CK(hipGraphLaunch(gfe, st));
    }
    CK(hipStreamSynchronize(st));
    const int R = 50;
    float ta = 0.f, tb = 0.f;
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < R; ++r) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ta, e0, e1));
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < R; ++r) CK(hipGraphLaunch(gfe, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&tb, e0, e1));
    printf("G=%d NK=%d: graph of %d kernels %.2f us per kernel node | one kernel, %d grid-barrier phases %.2f us per phase\n",
           G, NK, NK, 1e3f * ta / R / NK, NK, 1e3f * tb / R / NK);
  }
  unsigned tk = 0;
  CK(hipMemcpy(&tk, ticket, sizeof(unsigned), hipMemcpyDeviceToHost));
  printf("ticket %u (expected %llu)\n", tk, (unsigned long long)G * NK * 210);
  return 0;
}
