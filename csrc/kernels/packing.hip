// Unpadded-step bookkeeping in one launch (gfx950).
//
// From the padded batch (mask, ids: [B, S]) build the packed layout the model runs on:
//   row_map[r]    padded position of packed row r (-1 for the bucket's filler rows)
//   cu[b]         first packed row of sequence b (cu[B] = real tokens)
//   ids_packed[r] token id of packed row r (filler rows repeat position 0's id)
// i.e. a stream compaction of the mask.  One 1024-thread workgroup scans the B*S flags in
// 4096-position chunks (wave prefix sums through DPP shuffles, wave totals through LDS),
// replacing the ~10 small library launches (nonzero_static = flag + block sums + scan +
// scatter, mask sum, cumsum, clamp, gather) it took in torch.  Reference: the padding
// the reference computes on (client1.py:38-45, padding='max_length').
#include "common.h"

namespace {

template <typename M, typename I>
__global__ __launch_bounds__(1024) void pack_kernel(const M* mask, const I* ids, int n, int S, int B, int rows,
                                                    int* row_map, int* cu, long long* ids_packed, int* step,
                                                    uint32_t* seed, long long* cls_rows, int* cls_rmap) {
  __shared__ int wsum[16];
  __shared__ int carry_s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) carry_s = 0;
  __syncthreads();
  for (int base = 0; base < n; base += 4096) {
    int f[4], local = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = base + 4 * tid + j;
      f[j] = (p < n && mask[p] != 0) ? 1 : 0;
      local += f[j];
    }
    // inclusive wave scan
    int incl = local;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int before = 0;
    for (int i = 0; i < w; ++i) before += wsum[i];
    const int carry = carry_s;
    int off = carry + before + incl - local;  // exclusive prefix of this thread's first position
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = base + 4 * tid + j;
      if (p < n && p % S == 0) {
        cu[p / S] = off;  // tokens before sequence p / S
        if (cls_rows) cls_rows[p / S] = off;  // (pruned last block: its [CLS] row, int64)
      }
      if (f[j]) {
        if (off < rows) {
          row_map[off] = p;
          ids_packed[off] = (long long)ids[p];
        }
        ++off;
      }
    }
    __syncthreads();  // every wave has read carry_s and wsum
    if (tid == 1023) carry_s = off;  // the last thread's running offset = new carry
    __syncthreads();
  }
  const int total = carry_s;
  if (tid == 0) {
    cu[B] = total;
    // the training step's counters (Adam step, dropout seed) ride on this launch instead of a
    // kernel of their own; nothing in this kernel reads them
    if (step) step[0] += 1;
    if (seed) seed[0] += 1;
  }
  const long long id0 = (long long)ids[0];
  for (int r = total + tid; r < rows; r += 1024) {
    row_map[r] = -1;
    ids_packed[r] = id0;
  }
  if (cls_rmap) {
    // pruned last block: the padded row whose dropout masks the kept row of sequence b uses --
    // that of packed row cu[b] (b * S, or, for an empty sequence, the row its [CLS] row belongs
    // to), exactly what the unpruned LayerNorms hash it by; filler rows act as padded row 0
    __syncthreads();  // row_map / cu of this block are written
    for (int b = tid; b < B; b += 1024) {
      const int r = cu[b];
      cls_rmap[b] = r < total && r < rows ? max(row_map[r], 0) : 0;
    }
  }
}

// Pruned last block (ops/functional.py LayerFn._forward_pruned): two [rows][D] bf16 matrices
// gathered at the same row list in one launch (out_i[k] = in_i[idx[k]]), and the reverse: two
// [n][D] matrices scattered into zero-filled [T][D] ones (out_i[idx[k]] = in_i[k] for k < nsrc,
// every other row 0).  One thread moves 16 bytes; the scatter finds a row's source by binary
// search over the non-decreasing idx[0, nsrc) (the [CLS] rows), so each output row is written once.
__global__ __launch_bounds__(256) void gather_rows2_kernel(const uint4* a, const uint4* b, uint4* oa, uint4* ob,
                                                           const long long* idx, int n, int d16) {
  const long long i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= (long long)n * d16) return;
  const long long r = i / d16, c = i - r * d16;
  const long long src = idx[r] * d16 + c;
  oa[i] = a[src];
  ob[i] = b[src];
}
constexpr int SCATTER_LDS_IDX = 512;
__global__ __launch_bounds__(256) void scatter_rows2_kernel(const uint4* a, const uint4* b, uint4* oa, uint4* ob,
                                                            const long long* idx, int nsrc, int T, int d16) {
  // the (short, ascending) source row list staged in LDS once per block: the per-element binary
  // search then costs LDS latency instead of dependent global loads
  __shared__ long long sidx[SCATTER_LDS_IDX];
  const bool lds = nsrc <= SCATTER_LDS_IDX;
  if (lds)
    for (int k = threadIdx.x; k < nsrc; k += 256) sidx[k] = idx[k];
  __syncthreads();
  // 32-bit index math (T * d16 < 2^31, checked by the launcher): a 64-bit division is a runtime
  // call with a scratch frame
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= T * d16) return;
  const int r = i / d16, c = i - r * d16;
  // LAST k with idx[k] == r: an empty sequence (all-zero mask row) repeats its successor's [CLS]
  // row cu[b] == cu[b+1], and -- as in head_bwd's last-owner rule -- the later sequence (the one
  // that actually owns the row) wins
  // (one search loop per address space: a select between the LDS and the global list made the
  //  pointer generic and cost the kernel a scratch frame)
  int lo = 0, hi = nsrc;  // first k with idx[k] > r
  bool hit;
  if (lds) {
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (sidx[mid] <= r) lo = mid + 1; else hi = mid;
    }
    hit = lo > 0 && sidx[lo - 1] == r;
  } else {
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (idx[mid] <= r) lo = mid + 1; else hi = mid;
    }
    hit = lo > 0 && idx[lo - 1] == r;
  }
  const int k = lo - 1;
  // (branches, not `hit ? a[..] : z`: hipcc turned that select into a load through a pointer to
  //  either the row or a stack copy of z -- flat loads and a scratch frame)
  if (hit) {
    oa[i] = a[(long long)k * d16 + c];
    ob[i] = b[(long long)k * d16 + c];
  } else {
    oa[i] = make_uint4(0, 0, 0, 0);
    ob[i] = make_uint4(0, 0, 0, 0);
  }
}

}  // namespace

extern "C" {

int fd_gather_rows2(const void* a, const void* b, void* oa, void* ob, const long long* idx, int n, int d_bytes,
                    hipStream_t st) {
  if (n <= 0 || d_bytes <= 0 || d_bytes % 16) return 1;
  const long long tot = (long long)n * (d_bytes / 16);
  hipLaunchKernelGGL(gather_rows2_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const uint4*)a,
                     (const uint4*)b, (uint4*)oa, (uint4*)ob, idx, n, d_bytes / 16);
  return 0;
}

int fd_scatter_rows2(const void* a, const void* b, void* oa, void* ob, const long long* idx, int nsrc, int T,
                     int d_bytes, hipStream_t st) {
  if (nsrc < 0 || T <= 0 || d_bytes <= 0 || d_bytes % 16) return 1;
  const long long tot = (long long)T * (d_bytes / 16);
  if (tot >= (1ll << 31)) return 1;
  hipLaunchKernelGGL(scatter_rows2_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const uint4*)a,
                     (const uint4*)b, (uint4*)oa, (uint4*)ob, idx, nsrc, T, d_bytes / 16);
  return 0;
}


// mask_bytes / ids_bytes: 8 (int64) or 4 (int32) / 1 (uint8 mask).  n = B * S <= 1 << 20.
int fd_pack(const void* mask, int mask_bytes, const void* ids, int ids_bytes, int B, int S, int rows, int* row_map,
            int* cu, long long* ids_packed, int* step, uint32_t* seed, long long* cls_rows, int* cls_rmap,
            hipStream_t st) {
  const int n = B * S;
  if (B <= 0 || S <= 0 || rows <= 0 || n > (1 << 20)) return 1;
#define FD_PACK(MT, IT)                                                                                        \
  hipLaunchKernelGGL((pack_kernel<MT, IT>), dim3(1), dim3(1024), 0, st, (const MT*)mask, (const IT*)ids, n, S, B, \
                     rows, row_map, cu, ids_packed, step, seed, cls_rows, cls_rmap)
  if (mask_bytes == 8 && ids_bytes == 8) FD_PACK(long long, long long);
  else if (mask_bytes == 8 && ids_bytes == 4) FD_PACK(long long, int);
  else if (mask_bytes == 4 && ids_bytes == 8) FD_PACK(int, long long);
  else if (mask_bytes == 4 && ids_bytes == 4) FD_PACK(int, int);
  else if (mask_bytes == 1 && ids_bytes == 8) FD_PACK(unsigned char, long long);
  else if (mask_bytes == 1 && ids_bytes == 4) FD_PACK(unsigned char, int);
  else return 2;
#undef FD_PACK
  return 0;
}

}  // extern "C"
