// Shared helpers for the gfx950 (CDNA4, MI355X) kernels of this framework.
//
// Conventions
//  * bf16 tensors are passed as raw uint16 bits (`bf16_t`), fp32 as float.
//  * Wave size is 64; every kernel uses 256-thread blocks (4 waves) unless noted.
//  * MFMA: v_mfma_f32_16x16x32_bf16.  Operand lane maps (gfx950):
//      A frag, lane l: A[row = l&15][k = 8*(l>>4) + j], j = 0..7
//      B frag, lane l: B[k = 8*(l>>4) + j][col = l&15]
//      C/D,   lane l: D[row = 4*(l>>4) + r][col = l&15], r = 0..3
//  * Dropout masks come from a stateless counter hash (`drop_keep`) of
//    (seed, element index / 2) so the backward pass regenerates them instead of
//    storing them; the same hash is reproduced in torch for the CPU reference.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

typedef uint16_t bf16_t;
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define DEV __device__ __forceinline__

DEV float bf2f(uint32_t h) { return __uint_as_float(h << 16); }

// Round-to-nearest-even fp32 -> bf16 (NaN kept quiet).
DEV uint32_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

// Two fp32 -> packed bf16x2 with round-to-nearest-even; hipcc lowers the
// __bf16 conversions to one v_cvt_pk_bf16_f32 on gfx950 (NaN stays NaN).
DEV uint32_t pack_bf2(float a, float b) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

DEV float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
DEV float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// ---------------------------------------------------------------- dropout hash
// lowbias32-style finaliser over (idx * golden + seed).  Mirrored bit-exactly by
// ops/dropout.py::keep_mask (torch int64 arithmetic) for the CPU reference.
DEV uint32_t hash32(uint32_t seed, uint32_t idx) {
  uint32_t x = idx * 0x9E3779B1u + seed;
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// One hash serves an element pair: element idx keeps iff its 16-bit half of
// hash32(seed, idx >> 1) (low half: even idx, high half: odd) >= threshold, threshold =
// round(p * 2^16) (0 => always keep).  Half the integer multiplies of a hash per element --
// the attention forward's softmax phase and the LN epilogues are VALU-bound on them.
DEV bool drop_keep(uint32_t seed, uint32_t idx, uint32_t threshold) {
  const uint32_t h = hash32(seed, idx >> 1);
  return ((idx & 1u) ? (h >> 16) : (h & 0xffffu)) >= threshold;
}
// Keep bits (bit e) of the NE elements idx0 .. idx0 + NE - 1; idx0 even, NE even: NE / 2 hashes.
template <int NE>
DEV uint32_t drop_keep_bits(uint32_t seed, uint32_t idx0, uint32_t threshold) {
  static_assert(NE % 2 == 0 && NE <= 32, "element pairs");
  uint32_t bits = 0u;
#pragma unroll
  for (int e = 0; e < NE; e += 2) {
    const uint32_t h = hash32(seed, (idx0 >> 1) + (uint32_t)(e >> 1));
    bits |= ((h & 0xffffu) >= threshold ? 1u : 0u) << e;
    bits |= ((h >> 16) >= threshold ? 1u : 0u) << (e + 1);
  }
  return bits;
}

// Exact-erf GELU (HF DistilBERT's activation) evaluated with Abramowitz-Stegun
// 7.1.26 for erfc (|error| <= 1.5e-7, far below bf16 resolution): one v_exp and
// one v_rcp instead of ocml erff's branchy polynomial.  The exp(-x^2/2) term is
// shared with the derivative's pdf.
DEV void gelu_parts(float x, float& cdf, float& pdf) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  const float e = __expf(-z * z);
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
  const float half_erfc = 0.5f * poly * e;  // 0.5 * erfc(|x| / sqrt(2))
  cdf = x >= 0.f ? 1.0f - half_erfc : half_erfc;
  pdf = 0.39894228040143268f * e;
}
DEV float gelu_erf(float x) {
  float c, p;
  gelu_parts(x, c, p);
  return x * c;
}
DEV float gelu_erf_grad(float x) {
  float c, p;
  gelu_parts(x, c, p);
  return fmaf(x, p, c);
}

DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// XCD-aware bijective remap of a linear workgroup id (cdna_hip_programming.md
// T1): blocks that share an L2 (same id % 8) get a contiguous range of logical
// tiles, so neighbouring tiles reuse operand panels from one XCD's L2.
DEV int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}
