// Microbenchmark: per-CU fill rate from an L2-resident working set, by load path (gfx950).
//
// Why: the one-round GEMMs' K loop runs at ~65-70 GB/s of operand bytes per CU with LDS-DMA
// (in-kernel stamps, profiles/r3_gemm_stamps_*.txt), which is what bounds them.  This measures
// what each path can move per CU when every CU streams at once from its XCD's L2:
//   0  global_load_lds_dwordx4 (LDS-DMA, 1 KiB per wave instruction), counted vmcnt
//   1  global_load_dwordx4 into VGPRs (xor-folded so nothing is dead)
//   2  global_load_dwordx4 + ds_write_b128 into LDS (register staging)
// Each block (one per CU) reads 1 KiB pieces of a 2 MiB window shared by the blocks of its XCD
// (blockIdx % 8), so after the first pass everything is an L2 hit.  Build + run:
//   hipcc --offload-arch=gfx950 -O3 -o build/l2_fill csrc/bench/l2_fill.hip && ./build/l2_fill
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef __attribute__((address_space(3))) void lds_void;
constexpr int WINDOW = 2 << 20;   // bytes per XCD window
constexpr int PIECE = 1024;       // bytes per wave instruction

__device__ __forceinline__ void glds16(const void* src, char* lds) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void*)lds);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
}

template <int MODE, int INFLIGHT>
__global__ __launch_bounds__(512) void fill_kernel(const char* buf, int passes, unsigned* sink) {
  __shared__ __attribute__((aligned(1024))) char lds[64 * 1024];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const char* win = buf + (size_t)(blockIdx.x % 8) * WINDOW;
  const int npieces = WINDOW / PIECE;
  const int start = (blockIdx.x / 8) * 37;  // blocks of one XCD start at different pieces
  uint4 acc = make_uint4(0, 0, 0, 0);
  const int total = passes * npieces;
  int issued = 0;
  for (int i = wid; i < total; i += nw, ++issued) {
    const int piece = (start + i) % npieces;
    if constexpr (MODE == 0) {
      const char* src = win + (size_t)piece * PIECE + lane * 16;
      char* dst = lds + ((issued % 48) * PIECE);
      glds16(src, dst);
      if (issued >= INFLIGHT) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFLIGHT) : "memory");
    } else {
      // 8 loads in flight per wave: one batch of 8 pieces, then consume
      uint4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int pc = (start + i + u * nw) % npieces;
        v[u] = *reinterpret_cast<const uint4*>(win + (size_t)pc * PIECE + lane * 16);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if constexpr (MODE == 1) {
          acc.x ^= v[u].x; acc.y ^= v[u].y; acc.z ^= v[u].z; acc.w ^= v[u].w;
        } else {
          *reinterpret_cast<uint4*>(lds + (((issued + u) % 48) * PIECE) + lane * 16) = v[u];
        }
      }
      i += 7 * nw;
      issued += 7;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (MODE == 1) {
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[blockIdx.x] = 1;
  } else if (threadIdx.x == 0 && lds[lane] == 0x7f && lds[4097] == 0x11) {
    sink[blockIdx.x] = 2;
  }
}

template <int MODE, int INFLIGHT>
double run(const char* buf, unsigned* sink, int blocks, int threads, int passes) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((fill_kernel<MODE, INFLIGHT>), dim3(blocks), dim3(threads), 0, 0, buf, 1, sink);  // warm L2
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL((fill_kernel<MODE, INFLIGHT>), dim3(blocks), dim3(threads), 0, 0, buf, passes, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double bytes = (double)blocks * passes * WINDOW;
  return bytes / (ms * 1e-3) / 1e9;  // GB/s aggregate
}

int main(int argc, char** argv) {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  char* buf;
  unsigned* sink;
  CHECK(hipMalloc(&buf, 8 * (size_t)WINDOW));
  CHECK(hipMemset(buf, 1, 8 * (size_t)WINDOW));
  CHECK(hipMalloc(&sink, 4096 * sizeof(unsigned)));
  const int passes = 8;
  std::printf("CUs %d; per-CU GB/s (aggregate TB/s) reading an L2-resident 2 MiB window per XCD\n", cus);
  for (int blocks : {cus, cus / 4, cus / 16}) {
    for (int threads : {256, 512}) {
      const double d4 = run<0, 4>(buf, sink, blocks, threads, passes);
      const double d12 = run<0, 12>(buf, sink, blocks, threads, passes);
      const double r = run<1, 0>(buf, sink, blocks, threads, passes);
      const double w = run<2, 0>(buf, sink, blocks, threads, passes);
      std::printf("blocks %4d x %3d thr: lds-dma(4 in flight/wave) %6.1f (%5.2f) | lds-dma(12) %6.1f (%5.2f) | "
                  "vgpr %6.1f (%5.2f) | vgpr+ds_write %6.1f (%5.2f)\n",
                  blocks, threads, d4 / blocks, d4 / 1e3, d12 / blocks, d12 / 1e3, r / blocks, r / 1e3, w / blocks,
                  w / 1e3);
    }
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(sink));
  return 0;
}
