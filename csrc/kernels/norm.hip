// LayerNorm (fused residual + dropout), embedding and column-reduction kernels.
//
// Reference math (HF DistilBERT via client1.py:61, eps = 1e-12):
//   embeddings : y = Dropout(LN(word[id] + pos[s]))
//   sa block   : y = LN(attn_out + x)
//   ffn block  : y = LN(Dropout(lin2_out) + h)
// One wave owns one 768-wide row (12 values / lane, loaded as 8-byte bf16x4
// chunks so a wave instruction moves 512 contiguous bytes); statistics in fp32.
// The backward recomputes the pre-LN sum from the saved inputs and the
// stateless dropout hash instead of storing it, writes the input gradient(s)
// in bf16, and emits per-block partial column sums for dgamma, dbeta and the
// producer's bias gradient, which `colsum` reduces in a fixed order
// (deterministic, no atomics).
#include "common.h"

#include <cstdlib>

namespace {

struct LnArgs {
  const bf16_t* x;      // primary input (dropout applies to it)
  const bf16_t* r;      // residual (nullable)
  const float* gamma;
  const float* beta;
  bf16_t* y;
  float* mean;
  float* rstd;
  int T, D;
  float eps;
  const uint32_t* seed_ptr;
  uint32_t site, thr;
  float dscale;
  // backward
  const bf16_t* dy;
  bf16_t* dz;           // grad of the pre-LN sum (residual grad)
  bf16_t* dx;           // grad of the primary input through dropout (nullable if no dropout)
  float* part;          // [gridDim.x][3][D]: dgamma, dbeta, dbias partials
  // packed (unpadded) rows: row -> row of the padded [B*S] layout, used only to index the
  // dropout hash so a packed batch draws exactly the padded batch's masks (nullable)
  const int* row_map;
  // backward: x already IS the pre-LN sum z (saved by the LayerNorm-fused GEMM), r unused;
  // the dropout mask is still re-drawn for dx
  int zin;
};

// Half-wave row layout for D = 768: 32 lanes own a row, lane hl holds columns
// 8*(hl + 32c) .. +7 for c = 0..2 (three 16-byte bf16x8 loads), so one wave
// moves two rows per instruction and row statistics reduce in 5 xor-shuffles.
constexpr int HL = 32, CH = 3;  // lanes per row, 8-wide chunks per lane (D = HL * CH * 8)

DEV float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DEV void unpack8(const uint4& u, float (&f)[8]) {
  f[0] = lo_bf(u.x); f[1] = hi_bf(u.x); f[2] = lo_bf(u.y); f[3] = hi_bf(u.y);
  f[4] = lo_bf(u.z); f[5] = hi_bf(u.z); f[6] = lo_bf(u.w); f[7] = hi_bf(u.w);
}
DEV uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
}

// z = dropout(x) + r for one lane's 24 elements of `row`; keep bits recorded (bit 8c+e).
DEV void ln_load_sum(const LnArgs& a, int row, int hl, bool drop, uint32_t seed, float (&z)[CH][8],
                     uint32_t& keep) {
#pragma clang fp contract(off)
  uint4 xv[CH], rv[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const size_t off = (size_t)row * a.D + 8 * (hl + HL * c);
    xv[c] = *reinterpret_cast<const uint4*>(a.x + off);
    if (a.r) rv[c] = *reinterpret_cast<const uint4*>(a.r + off);
  }
  keep = 0xffffffu;
  const size_t hrow = a.row_map ? (size_t)(unsigned)a.row_map[row] : (size_t)row;  // dropout-hash row
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const size_t off = hrow * a.D + 8 * (hl + HL * c);
    unpack8(xv[c], z[c]);
    if (drop) {
      const uint32_t kb = drop_keep_bits<8>(seed, (uint32_t)off, a.thr);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool k = (kb >> e) & 1u;
        if (!a.zin) z[c][e] = k ? z[c][e] * a.dscale : 0.f;
        if (!k) keep &= ~(1u << (8 * c + e));
      }
    }
    if (a.r) {
      float rr[8];
      unpack8(rv[c], rr);
#pragma unroll
      for (int e = 0; e < 8; ++e) z[c][e] += rr[e];
    }
  }
}

__global__ __launch_bounds__(256) void ln_fwd_kernel(LnArgs a) {
  const int lane = threadIdx.x & 63, hl = lane & (HL - 1);
  const int row = blockIdx.x * 8 + (threadIdx.x >> 5);
  if (row >= a.T) return;  // whole half-waves exit together (T rows, 2 per wave)
  const bool drop = a.thr != 0;
  const uint32_t seed = drop ? hash32(a.seed_ptr[0], a.site) : 0u;
  // gamma / beta are fetched before the row data so their round trip overlaps it (issued
  // after the mean reduction they added two dependent memory round trips to the kernel).
  float4 gb[CH][4];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = 8 * (hl + HL * c);
    gb[c][0] = *reinterpret_cast<const float4*>(a.gamma + col);
    gb[c][1] = *reinterpret_cast<const float4*>(a.gamma + col + 4);
    gb[c][2] = *reinterpret_cast<const float4*>(a.beta + col);
    gb[c][3] = *reinterpret_cast<const float4*>(a.beta + col + 4);
  }
  float z[CH][8];
  uint32_t keep;
  ln_load_sum(a, row, hl, drop, seed, z, keep);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) s += z[c][e];
  const float mean = half_sum(s) / a.D;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float d = z[c][e] - mean; q += d * d; }
  const float rstd = rsqrtf(half_sum(q) / a.D + a.eps);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = 8 * (hl + HL * c);
    const float4 g0 = gb[c][0], g1 = gb[c][1], b0 = gb[c][2], b1 = gb[c][3];
    const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    float y[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) y[e] = (z[c][e] - mean) * rstd * g[e] + b[e];
    *reinterpret_cast<uint4*>(a.y + (size_t)row * a.D + col) = pack8(y);
  }
  if (hl == 0) { a.mean[row] = mean; a.rstd[row] = rstd; }
}

// Block-level reduction of per-lane column partials (NC*4 columns per lane,
// 4 waves) into part[blockIdx.x][which][D].
template <int NC>
DEV void block_colsum(float (&acc)[NC][4], float* lds, float* out, int D) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) lds[w * D + 4 * (lane + 64 * c) + e] = acc[c][e];
  __syncthreads();
  for (int col = threadIdx.x; col < D; col += blockDim.x) {
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += lds[i * D + col];
    out[col] = s;
  }
  __syncthreads();
}

// LayerNorm backward of one half-wave row from its output gradient dyv and pre-LN sum z (in xh,
// replaced by xhat): dz, dx (dropout), and this lane's dgamma / dbeta / dbias partials.  Shared by
// ln_bwd_kernel and head_ln_bwd_kernel with contraction off, so both round every product and sum
// the same way (the fused head launch's LayerNorm backward is bitwise ln_bwd_kernel's).
DEV void ln_bwd_row(const LnArgs& a, int row, int hl, bool drop, const float4 (&gm)[CH][2], const float (&dyv)[CH][8],
                    float (&xh)[CH][8], uint32_t keep, float mean, float rstd, float (&dg)[CH][8],
                    float (&db)[CH][8], float (&dbias)[CH][8]) {
#pragma clang fp contract(off)
  const int D = a.D;
  float gd[CH][8];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const float4 g0 = gm[c][0], g1 = gm[c][1];
    const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      xh[c][e] = (xh[c][e] - mean) * rstd;
      gd[c][e] = g[e] * dyv[c][e];
      s1 += gd[c][e];
      s2 += gd[c][e] * xh[c][e];
    }
  }
  s1 = half_sum(s1) / D;
  s2 = half_sum(s2) / D;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const size_t off = (size_t)row * D + 8 * (hl + HL * c);
    float dz[8], dx[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      dz[e] = rstd * (gd[c][e] - s1 - xh[c][e] * s2);
      dx[e] = ((keep >> (8 * c + e)) & 1u) ? dz[e] * (drop ? a.dscale : 1.f) : 0.f;
      dg[c][e] += dyv[c][e] * xh[c][e];
      db[c][e] += dyv[c][e];
      dbias[c][e] += dx[e];
    }
    *reinterpret_cast<uint4*>(a.dz + off) = pack8(dz);
    if (drop && a.dx) *reinterpret_cast<uint4*>(a.dx + off) = pack8(dx);
  }
}

// 16 rows per 512-thread block per iteration (two per wave); per-lane column
// partials for dgamma / dbeta / producer-bias, folded across the two half-waves
// and the 8 waves into part[blockIdx.x][3][D] (fixed order: deterministic).
__global__ __launch_bounds__(512) void ln_bwd_kernel(LnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [8 waves][D]
  const int lane = threadIdx.x & 63, hl = lane & (HL - 1), w = threadIdx.x >> 6;
  const int D = a.D;
  const bool drop = a.thr != 0;
  const uint32_t seed = drop ? hash32(a.seed_ptr[0], a.site) : 0u;
  float dg[CH][8] = {}, db[CH][8] = {}, dbias[CH][8] = {};
  // gamma and the row statistics are fetched ahead of the row data (after the data wait
  // they cost a second dependent round trip per row)
  float4 gm[CH][2];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = 8 * (hl + HL * c);
    gm[c][0] = *reinterpret_cast<const float4*>(a.gamma + col);
    gm[c][1] = *reinterpret_cast<const float4*>(a.gamma + col + 4);
  }
  const int rows_per_iter = (blockDim.x >> 5);
  for (int row = blockIdx.x * rows_per_iter + (threadIdx.x >> 5); row < a.T; row += gridDim.x * rows_per_iter) {
    const float mean = a.mean[row], rstd = a.rstd[row];
    uint4 dv[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c)
      dv[c] = *reinterpret_cast<const uint4*>(a.dy + (size_t)row * D + 8 * (hl + HL * c));
    float xh[CH][8];
    uint32_t keep;
    ln_load_sum(a, row, hl, drop, seed, xh, keep);
    float dyv[CH][8];
#pragma unroll
    for (int c = 0; c < CH; ++c) unpack8(dv[c], dyv[c]);
    ln_bwd_row(a, row, hl, drop, gm, dyv, xh, keep, mean, rstd, dg, db, dbias);
  }
  // fold the two half-waves (same columns, different rows), then the 8 waves
  float* out = a.part + (size_t)blockIdx.x * 3 * D;
  float (*accs[3])[8] = {dg, db, dbias};
#pragma unroll
  for (int which = 0; which < 3; ++which) {
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) accs[which][c][e] += __shfl_xor(accs[which][c][e], 32, 64);
    if (lane < HL) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        float* dst = lds + w * D + 8 * (hl + HL * c);
        *reinterpret_cast<float4*>(dst) =
            make_float4(accs[which][c][0], accs[which][c][1], accs[which][c][2], accs[which][c][3]);
        *reinterpret_cast<float4*>(dst + 4) =
            make_float4(accs[which][c][4], accs[which][c][5], accs[which][c][6], accs[which][c][7]);
      }
    }
    __syncthreads();
    const int nw = blockDim.x >> 6;
    for (int col = threadIdx.x; col < D; col += blockDim.x) {
      float sum = 0.f;
      for (int i = 0; i < nw; ++i) sum += lds[i * D + col];
      out[which * D + col] = sum;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ embeddings
struct EmbArgs {
  const void* ids;   // int64 or int32 [T]
  int ids64;
  const bf16_t* word;
  const bf16_t* pos;
  const float* gamma;
  const float* beta;
  bf16_t* y;
  float* mean;
  float* rstd;
  int T, S, D;
  float eps;
  const uint32_t* seed_ptr;
  uint32_t site, thr;
  float dscale;
  const bf16_t* dy;
  float* dz;       // fp32 [T][D]
  float* part;     // [grid][2][D]
  // packed rows (unpadded step): row -> padded row (position = padded row % S, dropout
  // hashed by the padded row; -1 = bucket filler, treated as padded row 0)
  const int* row_map;
  // forward only (nullable): the LayerNorm-fused GEMMs' exchange epoch (gemm.hip ln_epilogue),
  // advanced once per model forward here -- the first kernel of every forward -- so the fused
  // LayerNorm launches of this forward / backward tag their row statistics with a fresh epoch
  int* ln_epoch;
  // with ln_epoch (nullable): the exchange's granule buffer ([ln_stats_n] 8-byte {tag, value}).
  // A granule tag is (epoch * FD_LN_XSITES + xsite + 1) mod 2^32, so it repeats every 2^25
  // epochs: when the epoch crosses such a multiple, block 0 zeroes every granule first (tag 0
  // matches no launch), so a row block's statistics left untouched since then can never pass
  // for fresh ones
  unsigned long long* ln_stats;
  long long ln_stats_n;
  // forward only (nullable): the word-gradient grouping of the backward (rank sort of ids) is
  // computed by extra blocks of the forward launch (sort_blocks of them, after the rows' blocks)
  long long* sorted;
  long long* perm;
  int sort_blocks;
  // backward only (nullable): the word-gradient row flags to clear ([V] bytes) before the tail
  // launch sets this step's (first write of a step's gradient)
  unsigned char* now_clear;
  int V;
};

DEV int padded_row(const EmbArgs& a, int row) { return a.row_map ? max(a.row_map[row], 0) : row; }

DEV long load_id(const EmbArgs& a, int t) {
  return a.ids64 ? reinterpret_cast<const long long*>(a.ids)[t] : reinterpret_cast<const int*>(a.ids)[t];
}

// Deterministic token grouping without a library sort: the sorted position of
// token t is the number of tokens with key (id, index) smaller than its own
// (a rank sort; O(T^2) compares but T <= 16k and every compare is an LDS
// broadcast).  4 threads per token each scan a quarter of the keys.
template <typename I>
DEV void rank_sort_block(const I* ids, int T, long long* sorted, long long* perm, int* keys, int blk) {
  // every load of a pass issued before its LDS stores (a plain copy loop waits for each id in
  // turn: ~11 dependent round trips for a bs32 batch); rows past T re-read id T - 1, not stored
  constexpr int U = 16;
  for (int i0 = threadIdx.x; i0 < T; i0 += 256 * U) {
    I v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ids[min(i0 + u * 256, T - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * 256 < T) keys[i0 + u * 256] = (int)v[u];
  }
  __syncthreads();
  // 16 tokens per block, 16 threads per token (grid = T/16 blocks: ~256 for a bs32 batch,
  // one per CU, instead of T/64 blocks that left 3/4 of the chip idle)
  const int t = blk * 16 + (threadIdx.x >> 4);
  const int part = threadIdx.x & 15;
  int cnt = 0;
  int my = 0;
  if (t < T) {
    my = keys[t];
    // the 16 threads of a token read adjacent 16-byte groups: one ds_read_b128 each,
    // 256 contiguous bytes per token (the wave's 4 tokens read the same bytes: broadcast)
    const int T4 = T & ~63;
    for (int j = 4 * part; j < T4; j += 64) {
      const int4 k = *reinterpret_cast<const int4*>(keys + j);
      cnt += (k.x < my) | ((k.x == my) & (j < t));
      cnt += (k.y < my) | ((k.y == my) & (j + 1 < t));
      cnt += (k.z < my) | ((k.z == my) & (j + 2 < t));
      cnt += (k.w < my) | ((k.w == my) & (j + 3 < t));
    }
    for (int j = T4 + part; j < T; j += 16) {
      const int k = keys[j];
      cnt += (k < my) | ((k == my) & (j < t));
    }
  }
  cnt += __shfl_xor(cnt, 1, 64);
  cnt += __shfl_xor(cnt, 2, 64);
  cnt += __shfl_xor(cnt, 4, 64);
  cnt += __shfl_xor(cnt, 8, 64);
  if (t < T && part == 0) {
    sorted[cnt] = my;
    perm[cnt] = t;
  }
}

template <typename I>
__global__ __launch_bounds__(256) void rank_sort_kernel(const I* ids, int T, long long* sorted, long long* perm) {
  extern __shared__ __attribute__((aligned(16))) int keys[];  // T ids
  rank_sort_block<I>(ids, T, sorted, perm, keys, blockIdx.x);
}

template <int NC>
__global__ __launch_bounds__(256) void emb_fwd_kernel(EmbArgs a) {
  if (a.sort_blocks && (int)blockIdx.x >= (int)gridDim.x - a.sort_blocks) {  // block-uniform
    extern __shared__ __attribute__((aligned(16))) int keys[];  // T ids
    const int blk = blockIdx.x - (gridDim.x - a.sort_blocks);
    if (a.ids64) rank_sort_block<long long>(reinterpret_cast<const long long*>(a.ids), a.T, a.sorted, a.perm, keys, blk);
    else rank_sort_block<int>(reinterpret_cast<const int*>(a.ids), a.T, a.sorted, a.perm, keys, blk);
    return;
  }
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (a.ln_epoch && blockIdx.x == 0) {  // (read by later launches only)
    const unsigned e = (unsigned)a.ln_epoch[0] + 1u;
    __syncthreads();  // every thread has read the old epoch before thread 0 replaces it
    if (a.ln_stats && (e & ((1u << 25) - 1u)) == 0u)
      for (long long i = threadIdx.x; i < a.ln_stats_n; i += 256) a.ln_stats[i] = 0ull;
    if (threadIdx.x == 0) a.ln_epoch[0] = (int)e;
  }
  if (row >= a.T) return;
  const int D = a.D;
  const long id = load_id(a, row);
  const int prow = padded_row(a, row);
  const int s = prow % a.S;
  const bool drop = a.thr != 0;
  const uint32_t seed = drop ? hash32(a.seed_ptr[0], a.site) : 0u;
  float z[NC][4], sum = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = 4 * (lane + 64 * c);
    const uint2 wv = *reinterpret_cast<const uint2*>(a.word + (size_t)id * D + col);
    const uint2 pv = *reinterpret_cast<const uint2*>(a.pos + (size_t)s * D + col);
    z[c][0] = lo_bf(wv.x) + lo_bf(pv.x); z[c][1] = hi_bf(wv.x) + hi_bf(pv.x);
    z[c][2] = lo_bf(wv.y) + lo_bf(pv.y); z[c][3] = hi_bf(wv.y) + hi_bf(pv.y);
    sum += z[c][0] + z[c][1] + z[c][2] + z[c][3];
  }
  const float mean = wave_sum(sum) / D;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) { const float d = z[c][e] - mean; q += d * d; }
  const float rstd = rsqrtf(wave_sum(q) / D + a.eps);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = 4 * (lane + 64 * c);
    const size_t off = (size_t)row * D + col;
    const float4 g = *reinterpret_cast<const float4*>(a.gamma + col);
    const float4 b = *reinterpret_cast<const float4*>(a.beta + col);
    float y[4] = {(z[c][0] - mean) * rstd * g.x + b.x, (z[c][1] - mean) * rstd * g.y + b.y,
                  (z[c][2] - mean) * rstd * g.z + b.z, (z[c][3] - mean) * rstd * g.w + b.w};
    if (drop) {
      const uint32_t kb = drop_keep_bits<4>(seed, (uint32_t)((size_t)prow * D + col), a.thr);
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = (kb >> e) & 1u ? y[e] * a.dscale : 0.f;
    }
    *reinterpret_cast<uint2*>(a.y + off) = make_uint2(pack_bf2(y[0], y[1]), pack_bf2(y[2], y[3]));
  }
  if (lane == 0) { a.mean[row] = mean; a.rstd[row] = rstd; }
}

template <int NC>
__global__ __launch_bounds__(512) void emb_bwd_kernel(EmbArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int D = a.D;
  const bool drop = a.thr != 0;
  const uint32_t seed = drop ? hash32(a.seed_ptr[0], a.site) : 0u;
  float dg[NC][4] = {}, db[NC][4] = {};
  const int nw = blockDim.x >> 6;
  if (a.now_clear)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < a.V; i += gridDim.x * blockDim.x) a.now_clear[i] = 0;
  for (int row = blockIdx.x * nw + w; row < a.T; row += gridDim.x * nw) {
    const long id = load_id(a, row);
    const int prow = padded_row(a, row);
    const int s = prow % a.S;
    const float mean = a.mean[row], rstd = a.rstd[row];
    float xh[NC][4], gd[NC][4], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = 4 * (lane + 64 * c);
      const size_t off = (size_t)row * D + col;
      const uint2 wv = *reinterpret_cast<const uint2*>(a.word + (size_t)id * D + col);
      const uint2 pv = *reinterpret_cast<const uint2*>(a.pos + (size_t)s * D + col);
      const float z[4] = {lo_bf(wv.x) + lo_bf(pv.x), hi_bf(wv.x) + hi_bf(pv.x), lo_bf(wv.y) + lo_bf(pv.y),
                          hi_bf(wv.y) + hi_bf(pv.y)};
      const uint2 dv = *reinterpret_cast<const uint2*>(a.dy + off);
      float d4[4] = {lo_bf(dv.x), hi_bf(dv.x), lo_bf(dv.y), hi_bf(dv.y)};
      if (drop) {
        const uint32_t kb = drop_keep_bits<4>(seed, (uint32_t)((size_t)prow * D + col), a.thr);
#pragma unroll
        for (int e = 0; e < 4; ++e) d4[e] = (kb >> e) & 1u ? d4[e] * a.dscale : 0.f;
      }
      const float4 g = *reinterpret_cast<const float4*>(a.gamma + col);
      const float g4[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xh[c][e] = (z[e] - mean) * rstd;
        gd[c][e] = g4[e] * d4[e];
        s1 += gd[c][e];
        s2 += gd[c][e] * xh[c][e];
        dg[c][e] += d4[e] * xh[c][e];
        db[c][e] += d4[e];
      }
    }
    s1 = wave_sum(s1) / D;
    s2 = wave_sum(s2) / D;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = 4 * (lane + 64 * c);
      float4 o;
      o.x = rstd * (gd[c][0] - s1 - xh[c][0] * s2);
      o.y = rstd * (gd[c][1] - s1 - xh[c][1] * s2);
      o.z = rstd * (gd[c][2] - s1 - xh[c][2] * s2);
      o.w = rstd * (gd[c][3] - s1 - xh[c][3] * s2);
      *reinterpret_cast<float4*>(a.dz + (size_t)row * D + col) = o;
    }
  }
  float* out = a.part + (size_t)blockIdx.x * 3 * D;
  block_colsum<NC>(dg, lds, out, D);
  block_colsum<NC>(db, lds, out + D, D);
}

// dpos[s][:] = sum_b dz[b*S + s][:] -- fixed order; all B loads of a column issued
// back to back.  Rows s >= S are handled by a memset (first write) on the host side.
// cu (packed rows): sequence b's position s is row cu[b] + s when s < its length; the
// padded layout's extra terms are exact zeros, so both layouts give the same sums.
// grid (S, D/256): a block sums one position over the batch for 64 float4 columns, its 4
// thread groups taking every 4th sequence (8 loads in flight each), combined in a fixed order.
// Rows s < S: position gradient (sum over sequences).  Rows S <= s (first write only): zero --
// those positions never occur.  Block (s, cy) of a (rows, gy) grid.
constexpr int PG_GROUPS = 4, PG_COLS = 64;  // per block: 64 float4 columns x 4 sequence groups
DEV void pos_grad_block(int s, int cy, int gy, const float* dz, float* dpos, int B, int S, int D, int accumulate,
                        const int* cu) {
  if (s >= S) {
    for (int col = cy * 256 + threadIdx.x; col < D; col += gy * 256) dpos[(size_t)s * D + col] = 0.f;
    return;
  }
  __shared__ int s_cu[257];
  __shared__ float4 red[PG_GROUPS][PG_COLS];
  if (cu)
    for (int b = threadIdx.x; b <= B && b < 257; b += 256) s_cu[b] = cu[b];
  __syncthreads();
  const int c4 = cy * PG_COLS + (threadIdx.x % PG_COLS), grp = threadIdx.x / PG_COLS;
  const bool live = c4 < D / 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int b0 = grp; b0 < B; b0 += PG_GROUPS * 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {  // this group's sequences b0, b0 + 4, ...: loads in flight together
      const int b = b0 + u * PG_GROUPS;
      long long row = -1;
      if (b < B) {
        if (!cu) row = (long long)b * S + s;
        else if (B < 257 && s < s_cu[b + 1] - s_cu[b]) row = (long long)s_cu[b] + s;
        else if (B >= 257 && s < cu[b + 1] - cu[b]) row = (long long)cu[b] + s;
      }
      v[u] = (row >= 0 && live) ? reinterpret_cast<const float4*>(dz + (size_t)row * D)[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
  }
  red[grp][threadIdx.x % PG_COLS] = acc;
  __syncthreads();
  if (grp == 0 && live) {
    float4 t = accumulate ? reinterpret_cast<const float4*>(dpos + (size_t)s * D)[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int g = 0; g < PG_GROUPS; ++g) {  // fixed order: deterministic
      const float4 r = red[g][threadIdx.x];
      t.x += r.x; t.y += r.y; t.z += r.z; t.w += r.w;
    }
    reinterpret_cast<float4*>(dpos + (size_t)s * D)[c4] = t;
  }
}

// Word-embedding gradient over tokens grouped by id (rank sort above).  Pass 1:
// one block per WCH (16) sorted positions; every thread loads its WCH rows x 3 columns
// up front, then walks the runs: a run contained in the chunk is written
// straight to dword, a piece of a run crossing a chunk boundary goes to
// piece[start].  Pass 2: the chunk holding a crossing run's first position adds
// that run's pieces in chunk order.  Every output row is written by exactly one
// block -> deterministic, atomic-free.
constexpr int WCH = 16;
DEV void word_row_store(float* dword, long long id, int col, float acc, bool add) {
  float* dst = dword + (size_t)id * 768 + col;
  *dst = add ? *dst + acc : acc;
}

DEV void word_pieces_block(int bx, const long long* sorted, const long long* perm, const float* dz, float* piece,
                          float* dword, int T, int accumulate, unsigned char* now, unsigned char* ever) {
  constexpr int D = 768;
  __shared__ long long sid[WCH + 2];
  __shared__ long long sperm[WCH];
  const int c0 = bx * WCH, c1 = min(T, c0 + WCH), n = c1 - c0;
  if (threadIdx.x < n) {
    sid[threadIdx.x + 1] = sorted[c0 + threadIdx.x];
    sperm[threadIdx.x] = perm[c0 + threadIdx.x];
  }
  if (threadIdx.x == 0) sid[0] = c0 > 0 ? sorted[c0 - 1] : -1;
  if (threadIdx.x == 1) sid[n + 1] = c1 < T ? sorted[c1] : -1;
  __syncthreads();
  float v[3][WCH];
#pragma unroll
  for (int i = 0; i < WCH; ++i)
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c][i] = i < n ? dz[(size_t)sperm[i] * D + threadIdx.x + 256 * c] : 0.f;
  float acc[3] = {0.f, 0.f, 0.f};
  int start = 0;
#pragma unroll
  for (int i = 0; i < WCH; ++i) {
    if (i < n) {
#pragma unroll
      for (int c = 0; c < 3; ++c) acc[c] += v[c][i];
      const long long id = sid[i + 1];
      if (sid[i + 2] != id || i + 1 == n) {  // piece [start, i] ends here
        const bool run_starts_here = sid[start] != id;        // sid[start] is the predecessor
        const bool run_ends_here = i + 1 < n || sid[n + 1] != id;
        if (run_starts_here && run_ends_here) {
          const bool add = accumulate && (now ? now[id] != 0 : true);
#pragma unroll
          for (int c = 0; c < 3; ++c) word_row_store(dword, id, threadIdx.x + 256 * c, acc[c], add);
          if (threadIdx.x == 0 && now) { now[id] = 1; ever[id] = 1; }
        } else {
#pragma unroll
          for (int c = 0; c < 3; ++c) piece[(size_t)(c0 + start) * D + threadIdx.x + 256 * c] = acc[c];
        }
        acc[0] = acc[1] = acc[2] = 0.f;
        start = i + 1;
      }
    }
  }
}

DEV void word_combine_block(int bx, const long long* sorted, const float* piece, float* dword, int T, int accumulate,
                           unsigned char* now, unsigned char* ever) {
  constexpr int D = 768;
  const int c0 = bx * WCH, c1 = min(T, c0 + WCH);
  if (c1 >= T || sorted[c1] != sorted[c1 - 1]) return;  // no run crosses this chunk's end
  // The crossing run's first position in this chunk (the run is a suffix of the chunk) and its
  // end, found by the whole block at once instead of walking the sorted ids one dependent load
  // at a time (a template word's run spans many chunks).
  const long long id = sorted[c1 - 1];
  __shared__ int s_cnt, s_end;
  if (threadIdx.x == 0) { s_cnt = 0; s_end = T; }
  __syncthreads();
  if ((int)threadIdx.x < c1 - c0 && sorted[c0 + threadIdx.x] == id) atomicAdd(&s_cnt, 1);
  for (int base = c1;; base += 256) {
    const int j = base + (int)threadIdx.x;
    if (j < T && sorted[j] != id) atomicMin(&s_end, j);
    __syncthreads();
    const bool done = s_end < T || base + 256 >= T;
    __syncthreads();
    if (done) break;
  }
  const int a = c1 - s_cnt;
  if (a == c0 && c0 > 0 && sorted[c0 - 1] == id) return;  // run started in an earlier chunk
  const bool add = accumulate && (now ? now[id] != 0 : true);
  const int npieces = (s_end - c1 + WCH - 1) / WCH;  // chunk starts c1, c1 + WCH, ... inside the run
  for (int col = threadIdx.x; col < D; col += 256) {
    float acc = piece[(size_t)a * D + col];
    for (int p0 = 0; p0 < npieces; p0 += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = p0 + u < npieces ? piece[(size_t)(c1 + (p0 + u) * WCH) * D + col] : 0.f;
#pragma unroll
      for (int u = 0; u < 16; ++u) acc += v[u];
    }
    word_row_store(dword, id, col, acc, add);
  }
  if (threadIdx.x == 0 && now) { now[id] = 1; ever[id] = 1; }
}

// out_k[j] = (acc ? out_k[j] : 0) + sum_blk part[blk][k][j]  for k < nout (fixed order).
// Block = 4 partial-groups x 64 columns.  Every thread issues all of its partial
// loads back to back (UNR in flight) before summing them in a fixed order, so the
// reduction is bandwidth- not latency-bound; groups combine through LDS.
template <int UNR>
DEV void colsum_block(int bx, int k, const float* part, int nblk, int stride_blk, int D, float* o0, float* o1,
                      float* o2, int accumulate) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int j = bx * 64 + lane;
  float* out = k == 0 ? o0 : (k == 1 ? o1 : o2);
  if (!out) return;
  float s = 0.f;
  if (j < D) {
    const float* p = part + k * D + j;
    for (int b0 = grp; b0 < nblk; b0 += 4 * UNR) {
      float v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int b = b0 + 4 * u;
        v[u] = b < nblk ? p[(size_t)b * stride_blk] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) s += v[u];
    }
  }
  red[grp][lane] = s;
  __syncthreads();
  if (grp == 0 && j < D) {
    const float t = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    out[j] = accumulate ? out[j] + t : t;
  }
}
template <int UNR>
__global__ __launch_bounds__(256) void colsum_kernel(const float* part, int nblk, int stride_blk, int D,
                                                     float* o0, float* o1, float* o2, int accumulate) {
  colsum_block<UNR>(blockIdx.x, blockIdx.y, part, nblk, stride_blk, D, o0, o1, o2, accumulate);
}

// Deferred column-sum finalisation: every bias / LayerNorm-affine gradient of the
// backward leaves its per-block partials in a slot of its own, and ONE launch at the
// end of the backward reduces all of them (instead of one small launch per producer).
// Same per-column fixed-order sum as colsum_kernel: bitwise identical results.
constexpr int COLSUM_MAXJ = 32;
struct ColsumJob {
  const float* part;
  float* out[3];
  int nblk, stride_blk, D, nout, accumulate;
};
struct ColsumBatch {
  ColsumJob j[COLSUM_MAXJ];
  int start[COLSUM_MAXJ + 1];  // first block of job i (blocks = ceil(D/64) * nout)
  int n;
};

template <int UNR>
DEV void colsum_batched_block(const ColsumBatch& cb, int bx) {
  __shared__ float red[4][64];
  int ji = 0;
  while (ji + 1 < cb.n && bx >= cb.start[ji + 1]) ++ji;
  const ColsumJob& jb = cb.j[ji];
  const int local = bx - cb.start[ji];
  const int cblk = (jb.D + 63) / 64;
  const int k = local / cblk;
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int j = (local - k * cblk) * 64 + lane;
  float* out = jb.out[k];
  float s = 0.f;
  if (j < jb.D) {
    const float* p = jb.part + k * jb.D + j;
    for (int b0 = grp; b0 < jb.nblk; b0 += 4 * UNR) {
      float v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int b = b0 + 4 * u;
        v[u] = b < jb.nblk ? p[(size_t)b * jb.stride_blk] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) s += v[u];
    }
  }
  red[grp][lane] = s;
  __syncthreads();
  if (grp == 0 && j < jb.D && out) {
    const float t = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    out[j] = jb.accumulate ? out[j] + t : t;
  }
}

// The embedding backward's tail in two launches (after emb_bwd_kernel): A = the word-gradient
// pieces (chunk blocks) beside the position gradient (pos blocks); B = the crossing runs'
// combine beside the LayerNorm dgamma / dbeta column sums of emb_bwd_kernel's partials.  Each
// launch's two block kinds touch disjoint outputs, so they need no order between them.
struct EmbTail {
  const long long* sorted;
  const long long* perm;
  const float* dz;
  float* piece;         // [T][768] (pieces of runs crossing a chunk boundary)
  const float* lnpart;  // [lnblk][3][D] (emb_bwd_kernel's dgamma / dbeta partials)
  float* dword;
  float* dpos;
  float* dgamma;
  float* dbeta;
  const int* cu;
  unsigned char* now;
  unsigned char* ever;
  int T, B, S, D, chunks, pos_gy, cs_gx, lnblk, acc_mode, accumulate;
  int pos_blocks;
  // the backward's deferred column sums (bias / LayerNorm-affine gradients of every block), run as
  // extra blocks of the A launch instead of a colsum_batched launch of their own (cs.n == 0: none)
  ColsumBatch cs;
};
__global__ __launch_bounds__(256) void emb_tail_a_kernel(EmbTail t) {
  const int bx = blockIdx.x;
  if (bx < t.chunks) {
    word_pieces_block(bx, t.sorted, t.perm, t.dz, t.piece, t.dword, t.T, t.acc_mode, t.now, t.ever);
    return;
  }
  const int r = bx - t.chunks;
  if (r >= t.pos_blocks) {
    colsum_batched_block<16>(t.cs, r - t.pos_blocks);
    return;
  }
  pos_grad_block(r / t.pos_gy, r % t.pos_gy, t.pos_gy, t.dz, t.dpos, t.B, t.S, t.D, t.accumulate, t.cu);
}
__global__ __launch_bounds__(256) void emb_tail_b_kernel(EmbTail t) {
  const int bx = blockIdx.x;
  if (bx < t.chunks) {
    word_combine_block(bx, t.sorted, t.piece, t.dword, t.T, t.acc_mode, t.now, t.ever);
    return;
  }
  const int r = bx - t.chunks;
  colsum_block<16>(r % t.cs_gx, r / t.cs_gx, t.lnpart, t.lnblk, 3 * t.D, t.D, t.dgamma, t.dbeta, nullptr,
                   t.accumulate);
}

// Column sums of a bf16 [T][N] matrix into per-block partials [grid][N] (bias grads).
__global__ __launch_bounds__(256) void colsum_bf16_partial_kernel(const bf16_t* x, int T, int N, int rows_per_blk,
                                                                  float* part) {
  const int c4 = (blockIdx.y * 256 + threadIdx.x) * 4;
  if (c4 >= N) return;
  const int r0 = blockIdx.x * rows_per_blk, r1 = min(T, r0 + rows_per_blk);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (int rb = r0; rb < r1; rb += 16) {
    uint2 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u)
      v[u] = rb + u < r1 ? *reinterpret_cast<const uint2*>(x + (size_t)(rb + u) * N + c4) : make_uint2(0, 0);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      s0 += lo_bf(v[u].x); s1 += hi_bf(v[u].x); s2 += lo_bf(v[u].y); s3 += hi_bf(v[u].y);
    }
  }
  *reinterpret_cast<float4*>(part + (size_t)blockIdx.x * N + c4) = make_float4(s0, s1, s2, s3);
}

// Many bf16 column-sum partial jobs in one launch (the per-layer qkv-bias partials of a whole
// backward, computed at its end from the dqkv tensors the all-layer dW launch keeps alive anyway):
// block b belongs to job j with start[j] <= b < start[j + 1]; within a job the blocks walk
// (row block, column chunk) exactly as colsum_bf16_partial_kernel's grid, with the same per-block
// arithmetic, so the partials -- and the finalised sums -- are bitwise the per-layer launches'.
constexpr int CSB_MAXJ = 16;
struct ColsumBf16Batch {
  const bf16_t* x[CSB_MAXJ];
  float* part[CSB_MAXJ];
  int T[CSB_MAXJ], N[CSB_MAXJ], start[CSB_MAXJ + 1];
  int n, rows;
};
__global__ __launch_bounds__(256) void colsum_bf16_partial_batched_kernel(ColsumBf16Batch cb) {
  int j = 0;
  while (j + 1 < cb.n && (int)blockIdx.x >= cb.start[j + 1]) ++j;  // block-uniform
  const int local = blockIdx.x - cb.start[j];
  const int N = cb.N[j], T = cb.T[j];
  const int nchunk = (N / 4 + 255) / 256;
  const int bx = local / nchunk, by = local % nchunk;
  const int c4 = (by * 256 + threadIdx.x) * 4;
  if (c4 >= N) return;
  const bf16_t* x = cb.x[j];
  const int r0 = bx * cb.rows, r1 = min(T, r0 + cb.rows);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (int rb = r0; rb < r1; rb += 16) {
    uint2 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u)
      v[u] = rb + u < r1 ? *reinterpret_cast<const uint2*>(x + (size_t)(rb + u) * N + c4) : make_uint2(0, 0);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      s0 += lo_bf(v[u].x); s1 += hi_bf(v[u].x); s2 += lo_bf(v[u].y); s3 += hi_bf(v[u].y);
    }
  }
  *reinterpret_cast<float4*>(cb.part[j] + (size_t)bx * N + c4) = make_float4(s0, s1, s2, s3);
}

template <int UNR>
__global__ __launch_bounds__(256) void colsum_batched_kernel(ColsumBatch cb) {
  colsum_batched_block<UNR>(cb, blockIdx.x);
}


// ------------------------------------------------------------------ pruned head + output-LN backward
// The [CLS]-pruned training step's head (ops/functional.py HeadFn, fold_head): ONE launch for what
// were three -- the head forward with its loss mean (head_fwd_mean_kernel), the head backward
// (head_bwd_kernel) and the last block's output-LayerNorm backward (ln_bwd_kernel on the pruned
// rows), with the upstream gradient of the loss known to be 1 (loss.backward(unit_grad)).
//   blocks [0, nlb): ln_bwd_kernel's row blocks (16 rows per 512-thread block, half-wave rows);
//     each wave first computes the logits / dlogits of its two rows (head_logits: the head
//     forward's own code), the half-wave rebuilds its row's head gradient dy = (d0 w0 + d1 w1) *
//     keep (head_dh, bf16 -- head_bwd_kernel's dhidden) and runs the LayerNorm backward on it.
//   blocks [nlb, nlb + D / 64): head_bwd_kernel's column work, two 32-column groups per block,
//     after every wave has computed the dlogits of B / 8 rows; the first of them also writes the
//     logits / row losses / dlogits and the loss mean (head_fwd_mean_kernel's outputs).
// Every value is computed by the same expressions as in the three kernels it replaces, over the
// same rows per lane, so the outputs are bitwise theirs.  Head row b is hidden row b (the pruned
// layout); rows in [B, T) are the filler rows (no head gradient).
#include "head_common.h"

struct HeadLnArgs {
  HeadArgs h;
  LnArgs ln;
  int nlb;
};

constexpr int HLB_COLS = 32, HLB_GROUPS = 8, HLB_ROWS = 8;  // head_bwd_kernel's column tiling

__global__ __launch_bounds__(512) void head_ln_bwd_kernel(HeadLnArgs args) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const HeadArgs& h = args.h;
  const LnArgs& a = args.ln;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int D = a.D;
  const bool hdrop = h.thr != 0;
  const uint32_t hseed = hdrop ? hash32(h.seed_ptr[0], h.site) : 0u;
  if ((int)blockIdx.x >= args.nlb) {
    // ---- head_bwd_kernel's column blocks (+ the head forward's outputs in the first one)
    const int cb = blockIdx.x - args.nlb;
    float* dl = lds;                        // [B][2] dlogits
    float* red = lds + 2 * ((h.B + 3) & ~3);  // [2 groups][2][8][32]
    float* rl = red + 2 * 2 * HLB_GROUPS * HLB_COLS;  // [B] row losses (block 0's loss mean)
    const int sub = threadIdx.x >> 8, t = threadIdx.x & 255;
    const int c = t % HLB_COLS, grp = t / HLB_COLS;
    const int col = cb * 2 * HLB_COLS + sub * HLB_COLS + c;
    const bool live = col < D;
    const int colc = live ? col : 0;
    // this thread's column of the first HLB_ROWS [CLS] rows it sums (all of them for B <= 64),
    // loaded beside the logits' loads
    float xpre[HLB_ROWS];
#pragma unroll
    for (int u = 0; u < HLB_ROWS; ++u) xpre[u] = bf2f(h.hidden[cls_row(h, min(grp + u * HLB_GROUPS, h.B - 1)) * D + colc]);
    for (int b = w; b < h.B; b += 32) {  // rows b, b + 8, b + 16, b + 24 of this wave, interleaved
      const int rows[4] = {b, b + 8 < h.B ? b + 8 : -1, b + 16 < h.B ? b + 16 : -1, b + 24 < h.B ? b + 24 : -1};
      // labels / teacher logits loaded beside the logits' operands (not behind the stores below)
      HeadRowIn in[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) in[r] = head_row_in(h, rows[r] < 0 ? 0 : rows[r]);
      float z0[4], z1[4];
      head_logits_n<4>(h, rows, lane, z0, z1);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (rows[r] < 0) continue;
        const int br = rows[r];
        float loss, d0, d1;
        head_loss_grad_in(h, in[r], z0[r], z1[r], loss, d0, d1);
        if (lane == 0) {
          dl[2 * br] = d0;
          dl[2 * br + 1] = d1;
          if (cb == 0) {
            rl[br] = loss;
            h.logits[2 * br] = z0[r];
            h.logits[2 * br + 1] = z1[r];
            h.row_loss[br] = loss;
            h.dlogits[2 * br] = d0;
            h.dlogits[2 * br + 1] = d1;
          }
        }
      }
    }
    __syncthreads();  // dlogits (and block 0's row losses) in LDS
    if (cb == 0 && w == 0) loss_mean(h, lane, rl);
    float g0 = 0.f, g1 = 0.f;
    for (int b0 = grp; b0 < h.B; b0 += HLB_GROUPS * HLB_ROWS) {
      float x[HLB_ROWS];
#pragma unroll
      for (int u = 0; u < HLB_ROWS; ++u) {
        const int b = min(b0 + u * HLB_GROUPS, h.B - 1);
        x[u] = b0 == grp ? xpre[u] : bf2f(h.hidden[cls_row(h, b) * D + colc]);
      }
#pragma unroll
      for (int u = 0; u < HLB_ROWS; ++u) {
        const int b = b0 + u * HLB_GROUPS;
        if (b >= h.B) break;
        const float d0 = dl[2 * b], d1 = dl[2 * b + 1];
        const bool keep = !hdrop || drop_keep(hseed, (uint32_t)(b * D + colc), h.thr);
        const float sc = hdrop ? (keep ? h.dscale : 0.f) : 1.f;
        const float xv = x[u] * sc;
        head_col_acc(g0, d0, xv);
        head_col_acc(g1, d1, xv);
      }
    }
    float* rd = red + sub * 2 * HLB_GROUPS * HLB_COLS;
    rd[(0 * HLB_GROUPS + grp) * HLB_COLS + c] = g0;
    rd[(1 * HLB_GROUPS + grp) * HLB_COLS + c] = g1;
    __syncthreads();
    if (grp < 2 && live) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < HLB_GROUPS; ++i) s += rd[(grp * HLB_GROUPS + i) * HLB_COLS + c];
      float* dst = h.dW + grp * D + col;
      *dst = h.accumulate ? *dst + s : s;
    }
    if (cb == 0 && threadIdx.x < 2) {
      float s = 0.f;
      for (int b = 0; b < h.B; ++b) s += dl[2 * b + threadIdx.x];
      h.db[threadIdx.x] = h.accumulate ? h.db[threadIdx.x] + s : s;
    }
    return;
  }
  // ---- ln_bwd_kernel's row blocks, dy from the head
  const int hl = lane & (HL - 1);
  const bool drop = a.thr != 0;
  const uint32_t seed = drop ? hash32(a.seed_ptr[0], a.site) : 0u;
  float dg[CH][8] = {}, db[CH][8] = {}, dbias[CH][8] = {};
  float4 gm[CH][2], w0v[CH][2], w1v[CH][2];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = 8 * (hl + HL * c);
    gm[c][0] = *reinterpret_cast<const float4*>(a.gamma + col);
    gm[c][1] = *reinterpret_cast<const float4*>(a.gamma + col + 4);
    w0v[c][0] = *reinterpret_cast<const float4*>(h.W + col);
    w0v[c][1] = *reinterpret_cast<const float4*>(h.W + col + 4);
    w1v[c][0] = *reinterpret_cast<const float4*>(h.W + D + col);
    w1v[c][1] = *reinterpret_cast<const float4*>(h.W + D + col + 4);
  }
  const int rows_per_iter = (blockDim.x >> 5);
  for (int base = blockIdx.x * rows_per_iter; base < a.T; base += args.nlb * rows_per_iter) {
    const int row = base + (threadIdx.x >> 5);
    const int rr = min(row, a.T - 1);
    // every load of the iteration in flight at once: this half-wave's row operands and the wave's
    // two head rows (whole-wave reductions: wave-uniform control flow)
    const int rA = base + 2 * w;
    const int rows[2] = {rA < h.B ? rA : -1, rA + 1 < h.B ? rA + 1 : -1};
    HeadLoads<2> hlo;
    head_logits_load<2>(h, rows, lane, hlo);
    const int mine = lane < HL ? 0 : 1;
    const HeadRowIn in = head_row_in(h, rows[mine] < 0 ? 0 : rows[mine]);
    const float mean = a.mean[rr], rstd = a.rstd[rr];
    const bool empty = rr < h.B && empty_seq(h, rr);
    float xh[CH][8];
    uint32_t keep;
    ln_load_sum(a, rr, hl, drop, seed, xh, keep);
    float z0[2] = {0.f, 0.f}, z1[2] = {0.f, 0.f};
    if (rows[0] >= 0) head_logits_finish<2>(h, rows, lane, hlo, z0, z1);
    float d0 = 0.f, d1 = 0.f;
    if (rows[mine] >= 0) {
      float loss;
      head_loss_grad_in(h, in, z0[mine], z1[mine], loss, d0, d1);
    }
    if (row >= a.T) continue;  // (whole half-waves)
    const bool grad_row = row < h.B && !empty;
    float dyv[CH][8];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int col0 = 8 * (hl + HL * c);
      const uint32_t kb = hdrop ? drop_keep_bits<8>(hseed, (uint32_t)(row * D + col0), h.thr) : 0xffu;
      const float wa[8] = {w0v[c][0].x, w0v[c][0].y, w0v[c][0].z, w0v[c][0].w,
                           w0v[c][1].x, w0v[c][1].y, w0v[c][1].z, w0v[c][1].w};
      const float wb[8] = {w1v[c][0].x, w1v[c][0].y, w1v[c][0].z, w1v[c][0].w,
                           w1v[c][1].x, w1v[c][1].y, w1v[c][1].z, w1v[c][1].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sc = hdrop ? (((kb >> e) & 1u) ? h.dscale : 0.f) : 1.f;
        dyv[c][e] = grad_row ? bf2f(head_dh(d0, d1, wa[e], wb[e], sc)) : 0.f;
      }
    }
    ln_bwd_row(a, row, hl, drop, gm, dyv, xh, keep, mean, rstd, dg, db, dbias);
  }
  // fold the two half-waves (same columns, different rows), then the 8 waves (ln_bwd_kernel)
  float* out = a.part + (size_t)blockIdx.x * 3 * D;
  float (*accs[3])[8] = {dg, db, dbias};
#pragma unroll
  for (int which = 0; which < 3; ++which) {
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) accs[which][c][e] += __shfl_xor(accs[which][c][e], 32, 64);
    if (lane < HL) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        float* dst = lds + w * D + 8 * (hl + HL * c);
        *reinterpret_cast<float4*>(dst) =
            make_float4(accs[which][c][0], accs[which][c][1], accs[which][c][2], accs[which][c][3]);
        *reinterpret_cast<float4*>(dst + 4) =
            make_float4(accs[which][c][4], accs[which][c][5], accs[which][c][6], accs[which][c][7]);
      }
    }
    __syncthreads();
    const int nw = blockDim.x >> 6;
    for (int col = threadIdx.x; col < D; col += blockDim.x) {
      float sum = 0.f;
      for (int i = 0; i < nw; ++i) sum += lds[i * D + col];
      out[which * D + col] = sum;
    }
    __syncthreads();
  }
}

constexpr int LN_GRID = 256;
constexpr int LN_BWD_THREADS = 512;
// LayerNorm backward: 512-thread blocks (16 rows per pass) on up to 256 blocks.  (256-thread
// blocks on up to 512 -- every CU for a packed ~2.7 k-row batch -- measured slower, 2.476 vs
// 2.448 ms/step: more partial rows for the batched colsum; removed, profiles/r1_ab_ln_bwd_wide_slower.txt.)
constexpr int LN_BWD_GRID_MAX = 512;
int ln_bwd_threads() { return LN_BWD_THREADS; }

}  // namespace

extern "C" {

int fd_ln_fwd(const void* x, const void* r, const float* gamma, const float* beta, void* y, float* mean,
              float* rstd, int T, int D, float eps, const uint32_t* seed_ptr, uint32_t site, uint32_t thr,
              float dscale, const int* row_map, hipStream_t st) {
  if (D != 768) return 1;
  LnArgs a{};
  a.x = (const bf16_t*)x; a.r = (const bf16_t*)r; a.gamma = gamma; a.beta = beta; a.y = (bf16_t*)y;
  a.mean = mean; a.rstd = rstd; a.T = T; a.D = D; a.eps = eps;
  a.seed_ptr = seed_ptr; a.site = site; a.thr = thr; a.dscale = dscale; a.row_map = row_map;
  hipLaunchKernelGGL(ln_fwd_kernel, dim3((T + 7) / 8), dim3(256), 0, st, a);
  return 0;
}

// Writes dz (and dx when dropout is active); gradients of gamma/beta/producer-bias
// go to dgamma/dbeta/dbias (nullable), first-write unless accumulate.
int fd_ln_bwd(const void* dy, const void* x, const void* r, const float* gamma, const float* mean,
              const float* rstd, void* dz, void* dx, float* dgamma, float* dbeta, float* dbias, float* work,
              int T, int D, const uint32_t* seed_ptr, uint32_t site, uint32_t thr, float dscale,
              int accumulate, const int* row_map, int defer, int* nblk_out, int zin, hipStream_t st) {
  if (D != 768 || (zin && r)) return 1;
  LnArgs a{};
  a.zin = zin;
  a.dy = (const bf16_t*)dy; a.x = (const bf16_t*)x; a.r = (const bf16_t*)r; a.gamma = gamma;
  a.mean = (float*)mean; a.rstd = (float*)rstd; a.dz = (bf16_t*)dz; a.dx = (bf16_t*)dx; a.part = work;
  a.T = T; a.D = D; a.seed_ptr = seed_ptr; a.site = site; a.thr = thr; a.dscale = dscale; a.row_map = row_map;
  const int thr_n = ln_bwd_threads(), rows = thr_n / 32;
  const int grid = std::min(thr_n == 256 ? LN_BWD_GRID_MAX : LN_GRID, (T + rows - 1) / rows);
  if (nblk_out) *nblk_out = grid;
  hipLaunchKernelGGL(ln_bwd_kernel, dim3(grid), dim3(thr_n), (thr_n / 64) * D * sizeof(float),
                     st, a);
  if (!defer) hipLaunchKernelGGL(colsum_kernel<16>, dim3((D + 63) / 64, 3), dim3(256), 0, st, work, grid, 3 * D, D, dgamma,
                     dbeta, dbias, accumulate);
  return 0;
}


// The pruned training step's head + output-LayerNorm backward in one launch (head_ln_bwd_kernel).
// Head: hidden [T][D] (head row b = row b, b < B), W [2][D], bias [2], labels [B], logits / dlogits
// [B][2], loss [1], row_loss [B], loss_acc (nullable), dW [2][D] / db [2] (first-write unless
// accumulate), own [B + 1] (nullable), teacher logits (nullable).  LayerNorm: z = the saved pre-LN sum
// [T][D], gamma, mean / rstd [T], dz / dx out [T][D] (dx nullable without dropout), part: the
// [*nblk_out][3][D] dgamma / dbeta / dbias partials (deferred column sums).  D == 768.
int fd_head_ln_bwd(const void* hidden, int B, int T, int D, const float* W, const float* bias,
                   const uint32_t* seed_ptr, uint32_t hsite, uint32_t hthr, float hdscale, const long long* labels,
                   float* logits, float* loss, float* dlogits, float* row_loss, float* loss_acc, float* dW, float* db,
                   int accumulate, const int* own, const float* tlogits, float kd_T, float kd_alpha, const void* z,
                   const float* gamma, const float* mean, const float* rstd, void* dz, void* dx, float* part,
                   uint32_t site, uint32_t thr, float dscale, const int* row_map, int* nblk_out, hipStream_t st) {
  if (D != 768 || B <= 0 || B > T || B > 1024 || !labels || !row_loss) return 1;
  if (tlogits && !(kd_T > 0.f)) return 3;
  HeadLnArgs x{};
  HeadArgs& h = x.h;
  h.hidden = (const bf16_t*)hidden; h.B = B; h.S = 1; h.D = D; h.W = W; h.bias = bias;
  h.seed_ptr = seed_ptr; h.site = hsite; h.thr = hthr; h.dscale = hdscale; h.labels = labels;
  h.logits = logits; h.loss = loss; h.dlogits = dlogits; h.row_loss = row_loss; h.loss_acc = loss_acc;
  h.dW = dW; h.db = db; h.accumulate = accumulate; h.cls = nullptr; h.T = T; h.own = own;
  h.tlogits = tlogits; h.kd_T = kd_T; h.kd_alpha = kd_alpha;
  LnArgs& a = x.ln;
  a.zin = 1;
  a.x = (const bf16_t*)z; a.gamma = gamma; a.mean = (float*)mean; a.rstd = (float*)rstd;
  a.dz = (bf16_t*)dz; a.dx = (bf16_t*)dx; a.part = part; a.T = T; a.D = D;
  a.seed_ptr = seed_ptr; a.site = site; a.thr = thr; a.dscale = dscale; a.row_map = row_map;
  const int rows = LN_BWD_THREADS / 32;
  x.nlb = std::min(LN_GRID, (T + rows - 1) / rows);  // = ln_bwd's grid: the same partial rows
  if (nblk_out) *nblk_out = x.nlb;
  const size_t smem = std::max<size_t>((LN_BWD_THREADS / 64) * D * sizeof(float),
                                       (2 * ((B + 3) & ~3) + 2 * 2 * HLB_GROUPS * HLB_COLS + B) * sizeof(float));
  hipLaunchKernelGGL(head_ln_bwd_kernel, dim3(x.nlb + D / (2 * HLB_COLS)), dim3(LN_BWD_THREADS), smem, st, x);
  return 0;
}

int fd_emb_fwd(const void* ids, int ids64, const void* word, const void* pos, const float* gamma,
               const float* beta, void* y, float* mean, float* rstd, int T, int S, int D, float eps,
               const uint32_t* seed_ptr, uint32_t site, uint32_t thr, float dscale, const int* row_map,
               int* ln_epoch, unsigned long long* ln_stats, long long ln_stats_n, long long* sorted,
               long long* perm, hipStream_t st) {
  if (D != 768) return 1;
  if ((sorted == nullptr) != (perm == nullptr) || (sorted && T > 16384)) return 2;
  if (ln_stats && (!ln_epoch || ln_stats_n <= 0)) return 3;
  EmbArgs a{};
  a.ln_epoch = ln_epoch;
  a.ln_stats = ln_stats;
  a.ln_stats_n = ln_stats_n;
  a.sorted = sorted; a.perm = perm;
  a.sort_blocks = sorted ? (T + 15) / 16 : 0;
  a.ids = ids; a.ids64 = ids64; a.word = (const bf16_t*)word; a.pos = (const bf16_t*)pos; a.gamma = gamma;
  a.beta = beta; a.y = (bf16_t*)y; a.mean = mean; a.rstd = rstd; a.T = T; a.S = S; a.D = D; a.eps = eps;
  a.seed_ptr = seed_ptr; a.site = site; a.thr = thr; a.dscale = dscale; a.row_map = row_map;
  hipLaunchKernelGGL(emb_fwd_kernel<3>, dim3((T + 3) / 4 + a.sort_blocks), dim3(256),
                     sorted ? (size_t)T * sizeof(int) : 0, st, a);
  return 0;
}

// Embedding backward.  sorted/perm: torch.sort of the flattened ids (int64).
// work must hold max(grid*3*D, T*D) floats; dz_buf T*D floats.
int fd_emb_bwd(const void* dy, const void* ids, int ids64, const long long* sorted, const long long* perm,
               const void* word, const void* pos, const float* gamma, const float* mean, const float* rstd,
               float* dword, float* dpos, float* dgamma, float* dbeta, float* dz_buf, float* work, int T, int S,
               int B, int P, int V, int D, const uint32_t* seed_ptr, uint32_t site, uint32_t thr, float dscale,
               int accumulate, unsigned char* now, unsigned char* ever, const int* row_map, const int* cu,
               int ncs, const float* const* cs_parts, float* const* cs_outs, const int* cs_nblk, const int* cs_stride,
               const int* cs_D, const int* cs_nout, const int* cs_acc, hipStream_t st) {
  if (D != 768) return 1;
  if (ncs < 0 || ncs > COLSUM_MAXJ) return 5;
  EmbArgs a{};
  a.dy = (const bf16_t*)dy; a.ids = ids; a.ids64 = ids64; a.word = (const bf16_t*)word;
  a.pos = (const bf16_t*)pos; a.gamma = gamma; a.mean = (float*)mean; a.rstd = (float*)rstd; a.dz = dz_buf;
  a.part = work; a.T = T; a.S = S; a.D = D; a.seed_ptr = seed_ptr; a.site = site; a.thr = thr; a.dscale = dscale;
  a.row_map = row_map;
  // work = [T][D] word-gradient pieces, then the [grid][3][D] LayerNorm partials
  a.part = work + (size_t)T * D;
  a.now_clear = !accumulate ? now : nullptr;  // (set again by the tail for this step's ids)
  a.V = V;
  const int grid = std::min(LN_GRID, (T + 7) / 8);
  hipLaunchKernelGGL(emb_bwd_kernel<3>, dim3(grid), dim3(LN_BWD_THREADS), (LN_BWD_THREADS / 64) * D * sizeof(float),
                     st, a);
  if (!accumulate && !now) hipMemsetAsync(dword, 0, (size_t)V * D * sizeof(float), st);
  EmbTail t{};
  t.sorted = sorted; t.perm = perm; t.dz = dz_buf; t.piece = work; t.lnpart = a.part;
  t.dword = dword; t.dpos = dpos; t.dgamma = dgamma; t.dbeta = dbeta; t.cu = cu; t.now = now; t.ever = ever;
  t.T = T; t.B = B; t.S = S; t.D = D;
  t.chunks = (T + WCH - 1) / WCH;
  t.pos_gy = (D / 4 + PG_COLS - 1) / PG_COLS;
  t.cs_gx = (D + 63) / 64;
  t.lnblk = grid;
  t.acc_mode = now ? accumulate : 1;
  t.accumulate = accumulate;
  const int pos_rows = !accumulate && P > S ? P : S;
  t.pos_blocks = pos_rows * t.pos_gy;
  int cs_blocks = 0;
  t.cs.n = ncs;
  for (int i = 0; i < ncs; ++i) {
    if (cs_nout[i] < 1 || cs_nout[i] > 3 || cs_D[i] <= 0) return 6;
    t.cs.j[i] = ColsumJob{cs_parts[i], {cs_outs[3 * i], cs_outs[3 * i + 1], cs_outs[3 * i + 2]}, cs_nblk[i],
                          cs_stride[i], cs_D[i], cs_nout[i], cs_acc[i]};
    t.cs.start[i] = cs_blocks;
    cs_blocks += ((cs_D[i] + 63) / 64) * cs_nout[i];
  }
  t.cs.start[ncs] = cs_blocks;
  hipLaunchKernelGGL(emb_tail_a_kernel, dim3(t.chunks + t.pos_blocks + cs_blocks), dim3(256), 0, st, t);
  hipLaunchKernelGGL(emb_tail_b_kernel, dim3(t.chunks + 2 * t.cs_gx), dim3(256), 0, st, t);
  return 0;
}

// out[N] (+)= column sums of bf16 x[T][N]; work >= ceil(T/rows)*N floats.
// Group token ids (int64/int32) by value: sorted ids + originating positions (int64).
int fd_rank_sort(const void* ids, int ids64, int T, long long* sorted, long long* perm, hipStream_t st) {
  if (T > 16384) return 1;
  const size_t lds = (size_t)T * sizeof(int);
  if (ids64)
    hipLaunchKernelGGL(rank_sort_kernel<long long>, dim3((T + 15) / 16), dim3(256), lds, st, (const long long*)ids, T,
                       sorted, perm);
  else
    hipLaunchKernelGGL(rank_sort_kernel<int>, dim3((T + 15) / 16), dim3(256), lds, st, (const int*)ids, T, sorted,
                       perm);
  return 0;
}

// defer: leave the [nblk][N] partials in `work` (finalised later by fd_colsum_batched); returns nblk.
int fd_colsum_bf16(const void* x, int T, int N, float* out, float* work, int accumulate, int defer, int* nblk_out,
                   hipStream_t st) {
  if (N % 4 != 0) return 1;
  const int rows = 32;
  const int nblk = (T + rows - 1) / rows;
  if (nblk_out) *nblk_out = nblk;
  hipLaunchKernelGGL(colsum_bf16_partial_kernel, dim3(nblk, (N / 4 + 255) / 256), dim3(256), 0, st,
                     (const bf16_t*)x, T, N, rows, work);
  if (!defer)
    hipLaunchKernelGGL(colsum_kernel<16>, dim3((N + 63) / 64, 1), dim3(256), 0, st, work, nblk, N, N, out,
                       (float*)nullptr, (float*)nullptr, accumulate);
  return 0;
}

// n bf16 [T_i][N_i] matrices -> per-32-row-block partials part_i [ceil(T_i / 32)][N_i], one launch.
int fd_colsum_bf16_batched(int n, const void* const* xs, const int* T, const int* N, float* const* parts,
                           hipStream_t st) {
  for (int base = 0; base < n; base += CSB_MAXJ) {
    ColsumBf16Batch cb{};
    cb.n = std::min(CSB_MAXJ, n - base);
    cb.rows = 32;
    int blocks = 0;
    for (int i = 0; i < cb.n; ++i) {
      const int g = base + i;
      if (N[g] <= 0 || N[g] % 4 != 0 || T[g] <= 0) return 1;
      cb.x[i] = (const bf16_t*)xs[g];
      cb.part[i] = parts[g];
      cb.T[i] = T[g];
      cb.N[i] = N[g];
      cb.start[i] = blocks;
      blocks += ((T[g] + 31) / 32) * ((N[g] / 4 + 255) / 256);
    }
    cb.start[cb.n] = blocks;
    hipLaunchKernelGGL(colsum_bf16_partial_batched_kernel, dim3(blocks), dim3(256), 0, st, cb);
  }
  return 0;
}

// parts[i]: [nblk[i]][stride[i]] partials, output k of job i = columns k*D .. k*D+D-1.
int fd_colsum_batched(int n, const float* const* parts, float* const* outs /* n x 3 */, const int* nblk,
                      const int* stride, const int* D, const int* nout, const int* accumulate, hipStream_t st) {
  for (int base = 0; base < n; base += COLSUM_MAXJ) {
    ColsumBatch cb{};
    cb.n = std::min(COLSUM_MAXJ, n - base);
    int blocks = 0;
    for (int i = 0; i < cb.n; ++i) {
      const int g = base + i;
      if (nout[g] < 1 || nout[g] > 3 || D[g] <= 0) return 1;
      cb.j[i] = ColsumJob{parts[g], {outs[3 * g], outs[3 * g + 1], outs[3 * g + 2]}, nblk[g], stride[g], D[g],
                          nout[g], accumulate[g]};
      cb.start[i] = blocks;
      blocks += ((D[g] + 63) / 64) * nout[g];
    }
    cb.start[cb.n] = blocks;
    hipLaunchKernelGGL(colsum_batched_kernel<16>, dim3(blocks), dim3(256), 0, st, cb);
  }
  return 0;
}

}  // extern "C"
