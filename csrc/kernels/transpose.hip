// Batched bf16 matrix transpose: dst[c][r] = src[r][c] for up to 32 matrices in
// one launch (the encoder weight matrices of a DistilBERT/BERT model).
//
// Purpose: the backward dX GEMM dx = dy W reads W [out][in] MN-major, whose
// LDS-DMA staging measured ~30 % slower than the K-major staging of the same
// GEMM on W^T (profiles/r1_gemm_diag_*: with the in-loop DMA removed the two
// run at the same speed).  Refreshing W^T once per step (85 MB read + 85 MB
// write for DistilBERT) lets every dX GEMM run as the faster "NT" kernel.
//
// 64x64 tiles through LDS (+2-element row pad -> conflict-free column reads);
// 16-byte global loads and stores on both sides.
#include "common.h"

namespace {

constexpr int MAXMAT = 32;

struct TransposeBatch {
  const bf16_t* src[MAXMAT];
  bf16_t* dst[MAXMAT];
  int rows[MAXMAT];
  int cols[MAXMAT];
  int tile_start[MAXMAT + 1];  // prefix sum of 64x64 tile counts
  int n;
};

__global__ __launch_bounds__(256) void transpose_batched_kernel(TransposeBatch b) {
  __shared__ bf16_t tile[64][64 + 2];
  const int t = blockIdx.x;
  int m = 0;
  while (m + 1 < b.n && t >= b.tile_start[m + 1]) ++m;
  const int R = b.rows[m], C = b.cols[m];
  const int local = t - b.tile_start[m];
  const int tiles_c = C / 64;
  const int r0 = (local / tiles_c) * 64, c0 = (local % tiles_c) * 64;
  const bf16_t* src = b.src[m];
  bf16_t* dst = b.dst[m];
  const int tid = threadIdx.x;
  // load: 64 rows x 8 chunks of 8 bf16 -> 512 chunks, 2 per thread
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = i * 256 + tid, r = id >> 3, c = (id & 7) * 8;
    const uint4 v = *reinterpret_cast<const uint4*>(src + (size_t)(r0 + r) * C + c0 + c);
    const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[r][c + j] = e[j];
  }
  __syncthreads();
  // store: dst rows = src columns
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = i * 256 + tid, c = id >> 3, r = (id & 7) * 8;
    uint4 v;
    uint16_t* e = reinterpret_cast<uint16_t*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = tile[r + j][c];
    *reinterpret_cast<uint4*>(dst + (size_t)(c0 + c) * R + r0 + r) = v;
  }
}

}  // namespace

extern "C" {

// srcs[i]: [rows[i]][cols[i]] bf16, dsts[i]: [cols[i]][rows[i]]; rows, cols multiples of 64.
int fd_transpose_batched(const void* const* srcs, void* const* dsts, const int* rows, const int* cols, int n,
                         hipStream_t st) {
  if (n <= 0) return 0;
  if (n > MAXMAT) return 1;
  TransposeBatch b{};
  b.n = n;
  b.tile_start[0] = 0;
  for (int i = 0; i < n; ++i) {
    if (rows[i] % 64 || cols[i] % 64 || rows[i] <= 0 || cols[i] <= 0) return 2;
    b.src[i] = (const bf16_t*)srcs[i];
    b.dst[i] = (bf16_t*)dsts[i];
    b.rows[i] = rows[i];
    b.cols[i] = cols[i];
    b.tile_start[i + 1] = b.tile_start[i] + (rows[i] / 64) * (cols[i] / 64);
  }
  hipLaunchKernelGGL(transpose_batched_kernel, dim3(b.tile_start[n]), dim3(256), 0, st, b);
  return 0;
}

}  // extern "C"
