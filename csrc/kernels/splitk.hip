// Split-K reduce + fused epilogues for the small-M GEMMs (the pruned last block's [CLS] rows).
//
// A GEMM with M <= 64 rows and one tile per 64 x 64 output block runs on a dozen CUs for the
// whole K loop (the pruned block's out-proj / FFN GEMMs took 9-26 us each, 93 us per step,
// profiles/r3_kernel_stats_v1_ln_xsite.txt).  Here the product is split over K into fp32 slabs
// [splits][M][N] (gemm.hip fd_gemm_f32_splits: 12-48 tiles x splits = one round of the chip,
// 1-3 K tiles per block), and ONE launch of this file sums the slabs in slab order (fixed:
// deterministic) and applies the epilogue the single-pass GEMM would have:
//   EPI_BF16 / EPI_BIAS / EPI_BIAS_GELU / EPI_GELU_BWD / EPI_ADD  -- elementwise (gemm.hip);
//   EPI_LN      z = dropout(acc + bias) + res (bf16), y = LN(z): as gemm.hip's EPI_LN epilogue;
//   EPI_LN_BWD  dy = acc + res -> dz, dx and per-row dgamma / dbeta / dbias partials (EPI_LN_BWD).
// Reference ops: the DistilBERT projections reached from client1.py:61.
#include "common.h"
#include "adam_epi.h"

namespace {

#include "head_common.h"

enum : int { SK_BF16 = 0, SK_BIAS = 1, SK_BIAS_GELU = 2, SK_GELU_BWD = 3, SK_ADD = 4, SK_LN = 6, SK_LN_BWD = 7 };

struct SkArgs {
  const float* slabs;   // [splits][M][N] fp32
  long long sstride;    // elements between slabs (>= M * N)
  int splits, M, N;
  const float* bias;    // BIAS / BIAS_GELU / LN
  bf16_t* C;            // output [M][N] bf16 (LN_BWD: dz)
  bf16_t* aux;          // BIAS_GELU: u out;  GELU_BWD: u in
  bf16_t* aux_out;      // GELU_BWD: gelu(u) out (nullable)
  const bf16_t* res;    // ADD / LN / LN_BWD residual
  float* colsum;        // GELU_BWD / ADD: [ceil(M / 32)][N] column partials of C (nullable)
  FdLnEpi ln;           // LN: gamma, beta, mean, rstd (out), z (out, nullable), dropout, row_map, eps
                        // LN_BWD: gamma, mean, rstd, z (in), dx (out), colpart [M][3][N] (out)
  FdSkHead hd;          // LN (hd.W != nullptr): the pruned step's head + the LayerNorm backward
};

// Sum of the split-K slabs at element offset i (8 consecutive fp32), slab order.  The loads of
// 8 slabs are issued together before any is summed (a dependent load per slab left 16 memory
// round trips in a row: 7 us for the 16-slab LayerNorm rows).
DEV void slab_sum8(const SkArgs& a, size_t i, float (&v)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = 0.f;
  constexpr int G = 8;
  for (int s0 = 0; s0 < a.splits; s0 += G) {
    float4 p[G], q[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int s = min(s0 + j, a.splits - 1);
      p[j] = *reinterpret_cast<const float4*>(a.slabs + s * a.sstride + i);
      q[j] = *reinterpret_cast<const float4*>(a.slabs + s * a.sstride + i + 4);
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
      if (s0 + j < a.splits) {
        v[0] += p[j].x; v[1] += p[j].y; v[2] += p[j].z; v[3] += p[j].w;
        v[4] += q[j].x; v[5] += q[j].y; v[6] += q[j].z; v[7] += q[j].w;
      }
    }
  }
}

DEV void unpack8bf(const uint4& u, float (&f)[8]) {
  f[0] = lo_bf(u.x); f[1] = hi_bf(u.x); f[2] = lo_bf(u.y); f[3] = hi_bf(u.y);
  f[4] = lo_bf(u.z); f[5] = hi_bf(u.z); f[6] = lo_bf(u.w); f[7] = hi_bf(u.w);
}
DEV uint4 pack8bf(const float (&f)[8]) {
  return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
}

// Elementwise epilogues: a 256-thread block owns 64 columns (8 lanes x 8) of 32 rows; the
// column partials of the bf16 output (GELU_BWD / ADD with colsum) are folded over the block's
// 32 rows in a fixed order into colsum[blockIdx.y][N].
template <int EPI>
__global__ __launch_bounds__(256) void sk_elem_kernel(SkArgs a) {
  __shared__ float red[32][64 + 4];
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int n = blockIdx.x * 64 + cl * 8;
  const int m = blockIdx.y * 32 + rl;
  float out[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool live = m < a.M;
  if (live) {
    const size_t i = (size_t)m * a.N + n;
    float v[8];
    slab_sum8(a, i, v);
    if constexpr (EPI == SK_BIAS || EPI == SK_BIAS_GELU) {
      const float4 b0 = *reinterpret_cast<const float4*>(a.bias + n);
      const float4 b1 = *reinterpret_cast<const float4*>(a.bias + n + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
      v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    }
    uint4 o;
    if constexpr (EPI == SK_BIAS_GELU) {
      // GELU on the bf16-rounded pre-activation, exactly what the backward re-reads
      const uint4 u = pack8bf(v);
      *reinterpret_cast<uint4*>(a.aux + i) = u;
      float uf[8], g[8];
      unpack8bf(u, uf);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = gelu_erf(uf[e]);
      o = pack8bf(g);
    } else if constexpr (EPI == SK_GELU_BWD) {
      const uint4 u = *reinterpret_cast<const uint4*>(a.aux + i);
      float uf[8];
      unpack8bf(u, uf);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= gelu_erf_grad(uf[e]);
      if (a.aux_out) {
        float g[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = gelu_erf(uf[e]);
        *reinterpret_cast<uint4*>(a.aux_out + i) = pack8bf(g);
      }
      o = pack8bf(v);
    } else if constexpr (EPI == SK_ADD) {
      float r[8];
      unpack8bf(*reinterpret_cast<const uint4*>(a.res + i), r);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += r[e];
      o = pack8bf(v);
    } else {
      o = pack8bf(v);
    }
    *reinterpret_cast<uint4*>(a.C + i) = o;
    unpack8bf(o, out);  // the sums are of the stored (bf16) values, like the GEMM's colsum epilogue
  }
  if constexpr (EPI == SK_GELU_BWD || EPI == SK_ADD) {
    if (a.colsum == nullptr) return;
#pragma unroll
    for (int e = 0; e < 8; ++e) red[rl][cl * 8 + e] = out[e];
    __syncthreads();
    if (threadIdx.x < 64) {
      float s = 0.f;
      for (int r = 0; r < 32; ++r) s += red[r][threadIdx.x];
      a.colsum[(size_t)blockIdx.y * a.N + blockIdx.x * 64 + threadIdx.x] = s;
    }
  }
}

// Block-wide sum over the 4 waves (fixed order: every thread gets bitwise the same value).
DEV float block_sum4(float v, float* lds) {
  v = wave_sum(v);
  __syncthreads();  // lds reuse across calls
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  return (lds[0] + lds[1]) + (lds[2] + lds[3]);
}

// The pruned step's head on output row m (a.hd, FdSkHead), inside the output-LayerNorm epilogue
// block of that row: the logits by one wave in head_logits_finish's lane / chunk order over the
// row's bf16 values staged in LDS, then the loss / dlogits (head_loss_grad_in), the head gradient
// of the row (head_dh, zero for rows >= B and empty sequences) and the LayerNorm backward of it
// (sk_ln_kernel<true>'s arithmetic).  Per-row partials of the head dW / db, the loss mean and the
// LayerNorm affine gradients go to the deferred column sums.  N == 768.
DEV void sk_head_row(const SkArgs& a, int m, int t, bool act, int n, const float (&yb)[8], const float (&z)[8],
                     float mean, float rstd, const float (&g)[8], uint32_t lseed, size_t hrow) {
  __shared__ __attribute__((aligned(16))) uint16_t ys[768];
  __shared__ float hs[4];
  __shared__ float red[4];
  __shared__ unsigned ticket_s;
  const FdSkHead& H = a.hd;
  const FdLnEpi& L = a.ln;
  const int N = a.N, lane = t & 63;
  HeadArgs h{};
  h.D = N; h.B = H.B; h.W = H.W; h.bias = H.bias; h.seed_ptr = H.seed_ptr; h.site = H.site; h.thr = H.thr;
  h.dscale = H.dscale; h.labels = H.labels; h.tlogits = H.tlogits; h.kd_T = H.kd_T; h.kd_alpha = H.kd_alpha;
  const bool hr = m < H.B;
  if (act) *reinterpret_cast<uint4*>(ys + n) = pack8bf(yb);
  __syncthreads();
  if (hr && t < 64) {
    const int b[1] = {m};
    const bf16_t* x[1] = {nullptr};
    const bool hdrop = H.thr != 0;
    const uint32_t hseed = hdrop ? hash32(H.seed_ptr[0], H.site) : 0u;
    const HeadRowIn in = head_row_in(h, m);
    float z0[1] = {0.f}, z1[1] = {0.f};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int col = 4 * lane + 256 * j;
      const uint2 xv[1] = {*reinterpret_cast<const uint2*>(ys + col)};
      const float4 w0 = *reinterpret_cast<const float4*>(H.W + col);
      const float4 w1 = *reinterpret_cast<const float4*>(H.W + N + col);
      head_logit_chunk<1>(h, b, x, col, hdrop, hseed, xv, w0, w1, z0, z1);
    }
    const float l0 = wave_sum(z0[0]) + H.bias[0], l1 = wave_sum(z1[0]) + H.bias[1];
    float loss, d0, d1;
    head_loss_grad_in(h, in, l0, l1, loss, d0, d1);
    if (lane == 0) {
      H.logits[2 * m] = l0;
      H.logits[2 * m + 1] = l1;
      H.dlogits[2 * m] = d0;
      H.dlogits[2 * m + 1] = d1;
      hs[0] = d0; hs[1] = d1; hs[2] = loss;
    }
  }
  __syncthreads();
  const float d0 = hr ? hs[0] : 0.f, d1 = hr ? hs[1] : 0.f;
  if (t == 0) {
    const float lv = hr ? hs[2] / H.B : 0.f;
    H.dbpart[2 * m] = d0;
    H.dbpart[2 * m + 1] = d1;
    // The batch loss inside this launch (valid as soon as the forward returns, not only after the
    // deferred column sums of the backward), without fences (an agent-scope release / acquire writes
    // back / invalidates the whole L2): the row loss goes out as a write-through (agent-scope) store
    // that this thread drains (vmcnt(0)) BEFORE it takes a ticket (relaxed, agent scope) -- ln2_send's
    // hand-off form -- so the block holding the launch's last ticket finds every row loss in place and
    // sums them (at the end of this function, after its own row's work).  The ticket is never reset:
    // graph replays just count on (the last block of a launch holds ticket % rows == rows - 1).
    __hip_atomic_store(H.lpart + m, lv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned done = __hip_atomic_fetch_add(H.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ticket_s = done;
  }
  const bool grad_row = hr && !(H.own && H.own[m] == H.own[m + 1]);
  const bool hdrop = H.thr != 0;
  const uint32_t hseed = hdrop ? hash32(H.seed_ptr[0], H.site) : 0u;
  float dy[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, xh[8], gd[8];
  float s1 = 0.f, s2 = 0.f;
  if (act) {
    float w0[8], w1[8];
    const float4 a0 = *reinterpret_cast<const float4*>(H.W + n), a1 = *reinterpret_cast<const float4*>(H.W + n + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(H.W + N + n), b1 = *reinterpret_cast<const float4*>(H.W + N + n + 4);
    w0[0] = a0.x; w0[1] = a0.y; w0[2] = a0.z; w0[3] = a0.w; w0[4] = a1.x; w0[5] = a1.y; w0[6] = a1.z; w0[7] = a1.w;
    w1[0] = b0.x; w1[1] = b0.y; w1[2] = b0.z; w1[3] = b0.w; w1[4] = b1.x; w1[5] = b1.y; w1[6] = b1.z; w1[7] = b1.w;
    const uint32_t kb = hdrop ? drop_keep_bits<8>(hseed, (uint32_t)(m * N + n), H.thr) : 0xffu;
    float hp0[8], hp1[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sc = hdrop ? (((kb >> e) & 1u) ? H.dscale : 0.f) : 1.f;
      dy[e] = grad_row ? bf2f(head_dh(d0, d1, w0[e], w1[e], sc)) : 0.f;
      // head dW rows: d * dropout(x) (head_bwd's product; its column sums then run deferred)
      const float xd = yb[e] * sc;
      hp0[e] = hr ? d0 * xd : 0.f;
      hp1[e] = hr ? d1 * xd : 0.f;
    }
    float* hp = H.hpart + (size_t)m * 2 * N + n;
    *reinterpret_cast<float4*>(hp) = make_float4(hp0[0], hp0[1], hp0[2], hp0[3]);
    *reinterpret_cast<float4*>(hp + 4) = make_float4(hp0[4], hp0[5], hp0[6], hp0[7]);
    *reinterpret_cast<float4*>(hp + N) = make_float4(hp1[0], hp1[1], hp1[2], hp1[3]);
    *reinterpret_cast<float4*>(hp + N + 4) = make_float4(hp1[4], hp1[5], hp1[6], hp1[7]);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      xh[e] = (z[e] - mean) * rstd;
      gd[e] = g[e] * dy[e];
      s1 += gd[e];
      s2 += gd[e] * xh[e];
    }
  }
  s1 = block_sum4(s1, red) / N;
  s2 = block_sum4(s2, red) / N;
  if (act) {
    const size_t i = (size_t)m * N + n;
    const bool drop = L.thr != 0;
    const uint32_t kb = drop ? drop_keep_bits<8>(lseed, (uint32_t)(hrow * N + n), L.thr) : 0xffu;
    float dz[8], dx[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      dz[e] = rstd * (gd[e] - s1 - xh[e] * s2);
      dx[e] = drop ? ((kb >> e) & 1u ? dz[e] * L.dscale : 0.f) : dz[e];
    }
    *reinterpret_cast<uint4*>(H.dz + i) = pack8bf(dz);
    if (drop && H.dx) *reinterpret_cast<uint4*>(H.dx + i) = pack8bf(dx);
    float* cp = H.colpart + (size_t)m * 3 * N + n;
    float gx[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) gx[e] = dy[e] * xh[e];
    *reinterpret_cast<float4*>(cp) = make_float4(gx[0], gx[1], gx[2], gx[3]);
    *reinterpret_cast<float4*>(cp + 4) = make_float4(gx[4], gx[5], gx[6], gx[7]);
    *reinterpret_cast<float4*>(cp + N) = make_float4(dy[0], dy[1], dy[2], dy[3]);
    *reinterpret_cast<float4*>(cp + N + 4) = make_float4(dy[4], dy[5], dy[6], dy[7]);
    *reinterpret_cast<float4*>(cp + 2 * N) = make_float4(dx[0], dx[1], dx[2], dx[3]);
    *reinterpret_cast<float4*>(cp + 2 * N + 4) = make_float4(dx[4], dx[5], dx[6], dx[7]);
  }
  // the launch's last row block: the batch loss (one wave: lane l sums rows l, l + 64, ... in that
  // order, then a fixed butterfly -- deterministic)
  const unsigned rows = gridDim.x, done = ticket_s;  // (written before this function's later barriers)
  if (done % rows == rows - 1 && t < 64) {
    float s = 0.f;
    for (unsigned r = lane; r < rows; r += 64) s += __hip_atomic_load(H.lpart + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s = wave_sum(s);
    if (lane == 0) *H.loss = s;
  }
}

// LayerNorm epilogues: one 256-thread block per row, thread t owns columns 8t .. 8t+7 (t < N / 8,
// N <= 2048).  Forward: the math of gemm.hip's ln_epilogue (z rounded to bf16 before the
// statistics; mean, then the centred sum of squares).  Backward: s1 = mean(gamma dy),
// s2 = mean(gamma dy xhat) over the row, and the row's dgamma / dbeta / dbias contributions
// go to colpart[row][3][N] (finalised by the deferred column-sum launch).
template <bool BWD>
__global__ __launch_bounds__(256) void sk_ln_kernel(SkArgs a) {
  __shared__ float lds[4];
  const int m = blockIdx.x, t = threadIdx.x, N = a.N;
  const FdLnEpi& L = a.ln;
  const bool act = t * 8 < N;
  const int n = act ? t * 8 : 0;
  const size_t i = (size_t)m * N + n;
  const bool drop = L.thr != 0;
  const uint32_t seed = drop ? hash32(L.seed_ptr[0], L.site) : 0u;
  const size_t hrow = (drop && L.row_map) ? (size_t)(unsigned)L.row_map[m] : (size_t)m;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, r[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (act) {
    slab_sum8(a, i, v);
    unpack8bf(*reinterpret_cast<const uint4*>(a.res + i), r);
    const float4 g0 = *reinterpret_cast<const float4*>(L.gamma + n), g1 = *reinterpret_cast<const float4*>(L.gamma + n + 4);
    g[0] = g0.x; g[1] = g0.y; g[2] = g0.z; g[3] = g0.w; g[4] = g1.x; g[5] = g1.y; g[6] = g1.z; g[7] = g1.w;
  }
  if constexpr (!BWD) {
    float z[8], yb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (act) {
      const float4 b0 = *reinterpret_cast<const float4*>(a.bias + n), b1 = *reinterpret_cast<const float4*>(a.bias + n + 4);
      const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      const uint32_t kb = drop ? drop_keep_bits<8>(seed, (uint32_t)(hrow * N + n), L.thr) : 0xffu;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = v[e] + b[e];
        if (drop) x = (kb >> e) & 1u ? x * L.dscale : 0.f;
        v[e] = x + r[e];
      }
      const uint4 zb = pack8bf(v);
      unpack8bf(zb, z);
      if (L.z) *reinterpret_cast<uint4*>(L.z + i) = zb;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) z[e] = 0.f;
    }
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s += z[e];
    const float mean = block_sum4(s, lds) / N;
    float q = 0.f;
    if (act) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = z[e] - mean; q += d * d; }
    }
    const float rstd = rsqrtf(block_sum4(q, lds) / N + L.eps);
    if (act) {
      const float4 b0 = *reinterpret_cast<const float4*>(L.beta + n), b1 = *reinterpret_cast<const float4*>(L.beta + n + 4);
      const float bt[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      float y[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) y[e] = (z[e] - mean) * rstd * g[e] + bt[e];
      *reinterpret_cast<uint4*>(a.C + i) = pack8bf(y);
      if (a.hd.W) unpack8bf(pack8bf(y), yb);  // (the head reads the stored bf16 values)
    }
    if (t == 0) { L.mean[m] = mean; L.rstd[m] = rstd; }
    if (a.hd.W) sk_head_row(a, m, t, act, n, yb, z, mean, rstd, g, seed, hrow);
  } else {
    const float mean = L.mean[m], rstd = L.rstd[m];
    float dy[8], xh[8], gd[8];
    float s1 = 0.f, s2 = 0.f;
    if (act) {
      float zz[8];
      unpack8bf(*reinterpret_cast<const uint4*>(L.z + i), zz);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dy[e] = v[e] + r[e];
        xh[e] = (zz[e] - mean) * rstd;
        gd[e] = g[e] * dy[e];
        s1 += gd[e];
        s2 += gd[e] * xh[e];
      }
    }
    s1 = block_sum4(s1, lds) / N;
    s2 = block_sum4(s2, lds) / N;
    if (act) {
      float dz[8], dx[8];
      const uint32_t kb = drop ? drop_keep_bits<8>(seed, (uint32_t)(hrow * N + n), L.thr) : 0xffu;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dz[e] = rstd * (gd[e] - s1 - xh[e] * s2);
        dx[e] = drop ? ((kb >> e) & 1u ? dz[e] * L.dscale : 0.f) : dz[e];
      }
      *reinterpret_cast<uint4*>(a.C + i) = pack8bf(dz);
      if (drop && L.dx) *reinterpret_cast<uint4*>(L.dx + i) = pack8bf(dx);
      // this row's column contributions: dgamma = dy xhat, dbeta = dy, dbias = dx
      float* cp = L.colpart + (size_t)m * 3 * N + n;
      float gx[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) gx[e] = dy[e] * xh[e];
      *reinterpret_cast<float4*>(cp) = make_float4(gx[0], gx[1], gx[2], gx[3]);
      *reinterpret_cast<float4*>(cp + 4) = make_float4(gx[4], gx[5], gx[6], gx[7]);
      *reinterpret_cast<float4*>(cp + N) = make_float4(dy[0], dy[1], dy[2], dy[3]);
      *reinterpret_cast<float4*>(cp + N + 4) = make_float4(dy[4], dy[5], dy[6], dy[7]);
      *reinterpret_cast<float4*>(cp + 2 * N) = make_float4(dx[0], dx[1], dx[2], dx[3]);
      *reinterpret_cast<float4*>(cp + 2 * N + 4) = make_float4(dx[4], dx[5], dx[6], dx[7]);
    }
  }
}

}  // namespace

extern "C" {

// Reduce `splits` fp32 slabs [splits][M][N] (stride sstride) and apply epilogue `epi` (codes of
// gemm.hip's Epi).  Elementwise: N % 64 == 0; colsum (GELU_BWD / ADD) gets ceil(M / 32) partial
// rows, returned through *colsum_blocks.  LN / LN_BWD: N % 8 == 0, N <= 2048; ln fields as for
// gemm.hip's gemm_ln_kernel (LN_BWD: colpart has M partial rows of [3][N]).  0 or an error code.
int fd_splitk_epilogue(int epi, const float* slabs, long long sstride, int splits, int M, int N, const float* bias,
                       void* C, void* aux, void* aux_out, const void* res, float* colsum, int* colsum_blocks,
                       const FdLnEpi* ln, const FdSkHead* hd, hipStream_t st) {
  if (M <= 0 || N <= 0 || splits <= 0 || sstride < (long long)M * N || !slabs || !C) return 1;
  SkArgs a{};
  a.slabs = slabs; a.sstride = sstride; a.splits = splits; a.M = M; a.N = N;
  a.bias = bias; a.C = (bf16_t*)C; a.aux = (bf16_t*)aux; a.aux_out = (bf16_t*)aux_out;
  a.res = (const bf16_t*)res; a.colsum = colsum;
  if (ln) a.ln = *ln;
  if (hd && hd->W) {  // the fused head: LayerNorm forward only, N = 768, every output buffer given
    if (epi != SK_LN || N != 768 || hd->B <= 0 || hd->B > M || !hd->labels || !hd->logits || !hd->dlogits ||
        !hd->dz || !hd->colpart || !hd->hpart || !hd->dbpart || !hd->lpart || !hd->loss || !hd->ticket ||
        !hd->bias || !hd->seed_ptr ||
        (ln && ln->thr && !hd->dx))
      return 8;
    a.hd = *hd;
  }
  if (colsum_blocks) *colsum_blocks = 0;
  if (epi == SK_LN || epi == SK_LN_BWD) {
    if (!ln || !res || N % 8 || N > 2048 || !ln->gamma || !ln->mean || !ln->rstd) return 2;
    if (epi == SK_LN && (!bias || !ln->beta)) return 2;
    if (epi == SK_LN_BWD && (!ln->z || !ln->colpart)) return 2;
    if (epi == SK_LN) hipLaunchKernelGGL(sk_ln_kernel<false>, dim3(M), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(sk_ln_kernel<true>, dim3(M), dim3(256), 0, st, a);
    return 0;
  }
  if (N % 64) return 3;
  const dim3 grid(N / 64, (M + 31) / 32);
  if (colsum && colsum_blocks) *colsum_blocks = (M + 31) / 32;
  switch (epi) {
    case SK_BF16: hipLaunchKernelGGL(sk_elem_kernel<SK_BF16>, grid, dim3(256), 0, st, a); break;
    case SK_BIAS:
      if (!bias) return 2;
      hipLaunchKernelGGL(sk_elem_kernel<SK_BIAS>, grid, dim3(256), 0, st, a);
      break;
    case SK_BIAS_GELU:
      if (!bias || !aux) return 2;
      hipLaunchKernelGGL(sk_elem_kernel<SK_BIAS_GELU>, grid, dim3(256), 0, st, a);
      break;
    case SK_GELU_BWD:
      if (!aux) return 2;
      hipLaunchKernelGGL(sk_elem_kernel<SK_GELU_BWD>, grid, dim3(256), 0, st, a);
      break;
    case SK_ADD:
      if (!res) return 2;
      hipLaunchKernelGGL(sk_elem_kernel<SK_ADD>, grid, dim3(256), 0, st, a);
      break;
    default: return 4;
  }
  return 0;
}

}  // extern "C"

extern "C" {
int fd_gemm_f32_splits(const void* A, const void* Bt, float* slabs, long long slab_elems, int M, int N, int K,
                       int lda, int ldb, int splits, int b_mn, hipStream_t st);

// Split-K NT GEMM with a fused epilogue: C = epi(A Bt^T) via fp32 slabs (workspace, >= splits x
// M x N floats; splits <= 0: auto).  Two launches.  Returns the split count, or a negative code.
// b_mn: Bt is the weight W [K][N] itself (C = epi(A W)), read MN-major.
int fd_gemm_splitk(int epi, const void* A, const void* Bt, int M, int N, int K, float* workspace,
                   long long workspace_elems, int splits, const float* bias, void* C, void* aux, void* aux_out,
                   const void* res, float* colsum, int* colsum_blocks, const FdLnEpi* ln, const FdSkHead* hd,
                   int b_mn, hipStream_t st) {
  if (hd && hd->W && (epi != SK_LN || N != 768)) return -18;  // (checked before anything launches)
  const int s = fd_gemm_f32_splits(A, Bt, workspace, workspace_elems, M, N, K, K, b_mn ? N : K, splits, b_mn, st);
  if (s <= 0) return s == 0 ? -9 : s;
  const int rc = fd_splitk_epilogue(epi, workspace, (long long)M * N, s, M, N, bias, C, aux, aux_out, res, colsum,
                                    colsum_blocks, ln, hd, st);
  return rc ? -10 - rc : s;
}
}  // extern "C"
