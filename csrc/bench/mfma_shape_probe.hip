// Which bf16 MFMA shape the GEMMs should issue on gfx950 (every GEMM runs
// v_mfma_f32_16x16x32_bf16).  Two measurements per shape, chip-wide (4 waves per CU, one per SIMD,
// 1024 blocks):
//  (a) "regs": back-to-back MFMAs on register operands (4 independent accumulators per wave);
//  (b) "lds":  the same MFMA count with every A / B fragment re-read from LDS by ds_read_b128 first,
//      as a GEMM K loop does (one 16 B read per operand per lane per MFMA: 16x16x32 consumes
//      16 x 32 bf16 = 1 KiB of A and of B per instruction, 32x32x16 consumes 32 x 16 = 1 KiB).
// Reports dense TFLOP/s.  FLOPs per instruction: 16x16x32 = 16384, 32x32x16 = 32768.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o _bin/mfma_shape_probe csrc/bench/mfma_shape_probe.hip
// Run:   mfma_shape_probe [iters=4096]   (both operand-data kinds, ramp and random)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

// operand values: rnd = 0 a slow ramp (few toggling bits), rnd = 1 uniform in [-1, 1) from a hash (the
// MFMA power, and so the sustained clock, depends on the data)
__device__ float operand(int rnd, int tid, int i, unsigned salt) {
  if (!rnd) return (salt == 1u ? 0.001f : 0.002f) * (salt == 1u ? tid + i : tid - i);
  unsigned h = (unsigned)(tid * 8 + i) * 2654435761u ^ (salt * 0x9e3779b9u);
  h ^= h >> 15; h *= 0x85ebca6bu; h ^= h >> 13;
  return (float)(h & 0xffffu) / 32768.f - 1.f;
}

template <bool LDS>
__global__ __launch_bounds__(256) void mfma16_kernel(float* out, int iters, int rnd) {
  __shared__ __attribute__((aligned(16))) char smem[256 * 16 * 2];
  const int tid = threadIdx.x;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)operand(rnd, tid, i, 1u);
    b[i] = (__bf16)operand(rnd, tid, i, 2u);
  }
  *reinterpret_cast<bf16x8*>(smem + tid * 16) = a;
  *reinterpret_cast<bf16x8*>(smem + 4096 + tid * 16) = b;
  __syncthreads();
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
  for (int it = 0; it < iters; ++it) {
    if constexpr (LDS) {
      a = *reinterpret_cast<volatile bf16x8*>(smem + ((tid + it) & 255) * 16);
      b = *reinterpret_cast<volatile bf16x8*>(smem + 4096 + ((tid + 3 * it) & 255) * 16);
    }
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c3, 0, 0, 0);
  }
  const f32x4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 256 + tid] = s[0] + s[1] + s[2] + s[3];
}

template <bool LDS>
__global__ __launch_bounds__(256) void mfma32_kernel(float* out, int iters, int rnd) {
  __shared__ __attribute__((aligned(16))) char smem[256 * 16 * 2];
  const int tid = threadIdx.x;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)operand(rnd, tid, i, 1u);
    b[i] = (__bf16)operand(rnd, tid, i, 2u);
  }
  *reinterpret_cast<bf16x8*>(smem + tid * 16) = a;
  *reinterpret_cast<bf16x8*>(smem + 4096 + tid * 16) = b;
  __syncthreads();
  f32x16 c0 = {}, c1 = {};
  // two 32x32x16 per iteration = the FLOPs of four 16x16x32; the LDS variants of both shapes read
  // one A and one B fragment per iteration, i.e. the same LDS bytes per FLOP
  for (int it = 0; it < iters; ++it) {
    if constexpr (LDS) {
      a = *reinterpret_cast<volatile bf16x8*>(smem + ((tid + it) & 255) * 16);
      b = *reinterpret_cast<volatile bf16x8*>(smem + 4096 + ((tid + 3 * it) & 255) * 16);
    }
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
  out[blockIdx.x * 256 + tid] = s;
}

template <typename K>
double run(K kern, float* out, int blocks, int iters, int rnd, double flops_per_iter_per_wave) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, rnd);  // warm-up
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, rnd);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  const double flops = 5.0 * blocks * 4.0 * iters * flops_per_iter_per_wave;
  return flops / (ms * 1e-3) / 1e12;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4096;
  const int blocks = 1024;  // 4 blocks per CU x 4 waves: 4 waves per SIMD
  float* out;
  CK(hipMalloc(&out, sizeof(float) * blocks * 256));
  const double f16 = 4.0 * 16 * 16 * 32 * 2;  // four 16x16x32 per iteration
  const double f32 = 2.0 * 32 * 32 * 16 * 2;  // two 32x32x16 per iteration
  printf("bf16 MFMA shape probe: %d blocks x 4 waves, %d iterations (dense TFLOP/s, chip-wide)\n", blocks, iters);
  for (int rnd = 0; rnd < 2; ++rnd) {
    const char* data = rnd ? "random" : "ramp  ";
    printf("  %s 16x16x32  regs %8.1f   lds %8.1f\n", data, run(mfma16_kernel<false>, out, blocks, iters, rnd, f16),
           run(mfma16_kernel<true>, out, blocks, iters, rnd, f16));
    printf("  %s 32x32x16  regs %8.1f   lds %8.1f\n", data, run(mfma32_kernel<false>, out, blocks, iters, rnd, f32),
           run(mfma32_kernel<true>, out, blocks, iters, rnd, f32));
  }
  CK(hipFree(out));
  return 0;
}
