// Classifier head helpers shared by head_optim.hip (head forward / backward launches) and
// norm.hip (the pruned training step's fused head + output-LayerNorm backward launch), so both
// compute the logits, losses and gradients with the same code: bitwise the same values.
// Included inside each file's anonymous namespace (needs common.h).
// Head (client1.py:57-64, :108): pooled = hidden[:, 0, :] -> Dropout(0.3) -> Linear(768, 2) ->
// CrossEntropy(mean); 2-class CE == BCE-with-logits on z1 - z0.
#pragma once

struct HeadArgs {
  const bf16_t* hidden;  // [B*S, D]
  int B, S, D;
  const float* W;        // [2, D] fp32 master
  const float* bias;     // [2]
  const uint32_t* seed_ptr;
  uint32_t site, thr;
  float dscale;
  const long long* labels;  // nullable
  float* logits;         // [B, 2]
  float* loss;           // [1]
  float* dlogits;        // [B, 2] (written when labels given)
  float* row_loss;       // [B] scratch
  // backward
  const float* dlog_in;  // [B, 2]
  const float* gscale;   // nullable: dlog_in is scaled by gscale[0] (upstream grad of a fused loss)
  float* dW;             // [2, D]
  float* db;             // [2]
  bf16_t* dhidden;       // [B*S, D]; only CLS rows written
  int accumulate;
  // packed (unpadded) rows: sequence b's [CLS] is row cls[b] of a [T, D] hidden (nullable:
  // padded layout, row b*S); rows are clamped to T-1
  const int* cls;
  int T;
  // packed sequence starts (int32 [B+1], nullable): sequence b is EMPTY (all-zero mask row) when
  // own[b] == own[b+1]; its [CLS] row is not its own (the next sequence's, or a filler row), so
  // the backward gives it no hidden-state gradient -- the same in the pruned layout (distinct
  // rows) as in the packed one (shared rows), ADVICE r2
  const int* own;
  // knowledge distillation (nullable): teacher logits [B, 2]; the row loss becomes
  // kd_alpha * CE(z, y) + (1 - kd_alpha) * T^2 * KL(softmax(t / T) || softmax(z / T))
  const float* tlogits;
  float kd_T, kd_alpha;
  // nullable: the mean loss is also added here (a device-side running sum, e.g. a benchmark's
  // loss over a graph-replayed loop, with no separate add launch per step)
  float* loss_acc;
};

DEV size_t cls_row(const HeadArgs& a, int b) {
  return a.cls ? (size_t)min(max(a.cls[b], 0), a.T - 1) : (size_t)b * a.S;
}

// Logits of NR rows b[r] (one wave, the rows' loads and chains interleaved; b[r] < 0: skipped).
// Every lane returns the same bits (the xor butterfly of wave_sum adds the same pairs in every
// lane).  Floating-point contraction is off in the head helpers: every kernel that inlines them
// then rounds each product and sum the same way -- the fused pruned head (norm.hip) is bitwise
// head_fwd_mean_kernel + head_bwd_kernel, whatever the surrounding code lets the compiler fuse.
// One 4-column chunk (col = 4 lane + 256 j) of NR rows' logit sums.
template <int NR>
DEV void head_logit_chunk(const HeadArgs& a, const int (&b)[NR], const bf16_t* const (&x)[NR], int col, bool drop,
                          uint32_t seed, const uint2 (&xv)[NR], const float4& w0, const float4& w1, float (&z0)[NR],
                          float (&z1)[NR]) {
#pragma clang fp contract(off)
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    float v[4] = {lo_bf(xv[r].x), hi_bf(xv[r].x), lo_bf(xv[r].y), hi_bf(xv[r].y)};
    if (drop) {
      const uint32_t kb = drop_keep_bits<4>(seed, (uint32_t)((b[r] < 0 ? 0 : b[r]) * a.D + col), a.thr);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (kb >> e) & 1u ? v[e] * a.dscale : 0.f;
    }
    z0[r] += v[0] * w0.x + v[1] * w0.y + v[2] * w0.z + v[3] * w0.w;
    z1[r] += v[0] * w1.x + v[1] * w1.y + v[2] * w1.z + v[3] * w1.w;
  }
}

// Logits of NR rows b[r] (one wave, the rows' loads and chains interleaved; b[r] < 0: skipped).
// Every lane returns the same bits (the xor butterfly of wave_sum adds the same pairs in every
// lane).  Floating-point contraction is off in the head helpers: every kernel that inlines them
// then rounds each product and sum the same way -- the fused pruned head (norm.hip) is bitwise
// head_fwd_mean_kernel + head_bwd_kernel, whatever the surrounding code lets the compiler fuse.
// D = 768 (DistilBERT / BERT-base): the three chunks' loads are all issued before the first sum
// (one memory round trip instead of three); other widths walk the chunks (same sums, same order).
// The loads of NR rows' logits at D = 768 (three 4-column chunks per lane), issued together so a
// caller can put them in flight beside its own loads before the first use (head_logits_finish).
template <int NR>
struct HeadLoads {
  uint2 xv[3][NR];
  float4 w0[3], w1[3];
};
template <int NR>
DEV void head_logits_load(const HeadArgs& a, const int (&b)[NR], int lane, HeadLoads<NR>& L) {
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int col = 4 * lane + 256 * j;
#pragma unroll
    for (int r = 0; r < NR; ++r)
      L.xv[j][r] = *reinterpret_cast<const uint2*>(a.hidden + cls_row(a, b[r] < 0 ? 0 : b[r]) * a.D + col);
    L.w0[j] = *reinterpret_cast<const float4*>(a.W + col);
    L.w1[j] = *reinterpret_cast<const float4*>(a.W + a.D + col);
  }
}
template <int NR>
DEV void head_logits_finish(const HeadArgs& a, const int (&b)[NR], int lane, const HeadLoads<NR>& L,
                            float (&z0)[NR], float (&z1)[NR]) {
  const bool drop = a.thr != 0;
  const uint32_t seed = drop ? hash32(a.seed_ptr[0], a.site) : 0u;
  const bf16_t* x[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    x[r] = nullptr;
    z0[r] = 0.f;
    z1[r] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j)
    head_logit_chunk<NR>(a, b, x, 4 * lane + 256 * j, drop, seed, L.xv[j], L.w0[j], L.w1[j], z0, z1);
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    z0[r] = wave_sum(z0[r]) + a.bias[0];
    z1[r] = wave_sum(z1[r]) + a.bias[1];
  }
}

// Logits of NR rows b[r] (one wave, the rows' loads and chains interleaved; b[r] < 0: skipped).
// Every lane returns the same bits (the xor butterfly of wave_sum adds the same pairs in every
// lane).  Floating-point contraction is off in the head helpers: every kernel that inlines them
// then rounds each product and sum the same way -- the fused pruned head (norm.hip) is bitwise
// head_fwd_mean_kernel + head_bwd_kernel, whatever the surrounding code lets the compiler fuse.
// D = 768 (DistilBERT / BERT-base): the three chunks' loads are all issued before the first sum
// (one memory round trip instead of three); other widths walk the chunks (same sums, same order).
template <int NR>
DEV void head_logits_n(const HeadArgs& a, const int (&b)[NR], int lane, float (&z0)[NR], float (&z1)[NR]) {
#pragma clang fp contract(off)
  if (a.D == 768) {
    HeadLoads<NR> L;
    head_logits_load<NR>(a, b, lane, L);
    head_logits_finish<NR>(a, b, lane, L, z0, z1);
    return;
  }
  const bool drop = a.thr != 0;
  const uint32_t seed = drop ? hash32(a.seed_ptr[0], a.site) : 0u;
  const bf16_t* x[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    x[r] = a.hidden + cls_row(a, b[r] < 0 ? 0 : b[r]) * a.D;
    z0[r] = 0.f;
    z1[r] = 0.f;
  }
  for (int col = 4 * lane; col < a.D; col += 256) {
    uint2 xv[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) xv[r] = *reinterpret_cast<const uint2*>(x[r] + col);
    const float4 w0 = *reinterpret_cast<const float4*>(a.W + col);
    const float4 w1 = *reinterpret_cast<const float4*>(a.W + a.D + col);
    head_logit_chunk<NR>(a, b, x, col, drop, seed, xv, w0, w1, z0, z1);
  }
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    z0[r] = wave_sum(z0[r]) + a.bias[0];
    z1[r] = wave_sum(z1[r]) + a.bias[1];
  }
}

DEV void head_logits(const HeadArgs& a, int b, int lane, float& z0, float& z1) {
  const int bb[1] = {b};
  float y0[1], y1[1];
  head_logits_n<1>(a, bb, lane, y0, y1);
  z0 = y0[0];
  z1 = y1[0];
}

// Row b's label and (distillation) teacher logits, loadable ahead of the logits' reductions.
struct HeadRowIn {
  int y;
  float t0, t1;
};
DEV HeadRowIn head_row_in(const HeadArgs& a, int b) {
  HeadRowIn r;
  r.y = (int)a.labels[b];
  r.t0 = a.tlogits ? a.tlogits[2 * b] : 0.f;
  r.t1 = a.tlogits ? a.tlogits[2 * b + 1] : 0.f;
  return r;
}

// Row loss and dlogits (before the 1/B of the mean) of a row from its logits and label / teacher
// logits (head_row_in).
DEV void head_loss_grad_in(const HeadArgs& a, const HeadRowIn& in, float z0, float z1, float& loss, float& d0,
                           float& d1) {
#pragma clang fp contract(off)
  const float mx = fmaxf(z0, z1);
  const float lse = mx + __logf(__expf(z0 - mx) + __expf(z1 - mx));
  const int y = in.y;
  const float p1 = __expf(z1 - lse), p0 = __expf(z0 - lse);
  loss = lse - (y ? z1 : z0);
  d0 = p0 - (y == 0);
  d1 = p1 - (y == 1);
  if (a.tlogits) {
    // soft term at temperature T (2 classes): log-softmax of z / T and t / T
    const float iT = 1.f / a.kd_T;
    const float s0 = z0 * iT, s1 = z1 * iT, t0 = in.t0 * iT, t1 = in.t1 * iT;
    const float ms = fmaxf(s0, s1), mt = fmaxf(t0, t1);
    const float ls = ms + __logf(__expf(s0 - ms) + __expf(s1 - ms));
    const float lt = mt + __logf(__expf(t0 - mt) + __expf(t1 - mt));
    const float lq0 = s0 - ls, lq1 = s1 - ls;   // student log-probs
    const float lp0 = t0 - lt, lp1 = t1 - lt;   // teacher log-probs
    const float pt0 = __expf(lp0), pt1 = __expf(lp1);
    const float kl = pt0 * (lp0 - lq0) + pt1 * (lp1 - lq1);
    const float al = a.kd_alpha, T2 = a.kd_T * a.kd_T;
    loss = al * loss + (1.f - al) * T2 * kl;
    // d/dz of T^2 KL(p_t || softmax(z / T)) = T (q - p_t)
    d0 = al * d0 + (1.f - al) * a.kd_T * (__expf(lq0) - pt0);
    d1 = al * d1 + (1.f - al) * a.kd_T * (__expf(lq1) - pt1);
  }
  d0 = d0 / a.B;
  d1 = d1 / a.B;
}
DEV void head_loss_grad(const HeadArgs& a, int b, float z0, float z1, float& loss, float& d0, float& d1) {
  head_loss_grad_in(a, head_row_in(a, b), z0, z1, loss, d0, d1);
}

// Row b's outputs from its logits (lane 0 writes): logits, and with labels the row loss and dlogits.
DEV void head_row_out(const HeadArgs& a, int b, int lane, float z0, float z1) {
  if (lane == 0) {
    a.logits[2 * b] = z0;
    a.logits[2 * b + 1] = z1;
    if (a.labels) {
      float loss, d0, d1;
      head_loss_grad(a, b, z0, z1, loss, d0, d1);
      a.row_loss[b] = loss;
      a.dlogits[2 * b] = d0;
      a.dlogits[2 * b + 1] = d1;
    }
  }
}

// Row b of the head (one wave): logits, and with labels the row loss and dlogits.
DEV void head_row(const HeadArgs& a, int b, int lane) {
  float z0, z1;
  head_logits(a, b, lane, z0, z1);
  head_row_out(a, b, lane, z0, z1);
}

// rl: the row losses (a.row_loss, or the caller's LDS copy of them -- same values, same order)
DEV void loss_mean(const HeadArgs& a, int lane, const float* rl = nullptr) {  // one wave; fixed order
  if (!rl) rl = a.row_loss;
  float s = 0.f;
  for (int b = lane; b < a.B; b += 64) s += rl[b];
  s = wave_sum(s);
  if (lane == 0) {
    a.loss[0] = s / a.B;
    if (a.loss_acc) a.loss_acc[0] += s / a.B;
  }
}

DEV bool empty_seq(const HeadArgs& a, int b) { return a.own && a.own[b] == a.own[b + 1]; }

// dhidden of [CLS] element (b, col): (d0 w0 + d1 w1) * keep-scale, rounded to bf16.
DEV uint32_t head_dh(float d0, float d1, float w0, float w1, float sc) {
#pragma clang fp contract(off)
  return f2bf((d0 * w0 + d1 * w1) * sc);
}

// One [CLS] row's contribution to the head weight gradient column: g += d * x.
DEV void head_col_acc(float& g, float d, float xv) {
#pragma clang fp contract(off)
  g += d * xv;
}
