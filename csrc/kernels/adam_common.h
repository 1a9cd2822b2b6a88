// Adam shared by every launch that applies it: the run-table / row-flag launches (head_optim.hip)
// and the blocks of the all-layer weight-gradient launch that finish the optimizer step beside its
// last tiles (gemm.hip).  ONE copy of the per-element arithmetic, contraction off, so every kernel
// that inlines it rounds identically (bitwise equal parameters whichever launch updates them).
// Included inside each file's anonymous namespace (needs common.h).
#pragma once

// The Adam update of one element (torch.optim.Adam / AdamW defaults: bias-corrected, eps outside
// the square root; step_size = lr / bc1, inv_sqrt_bc2 = 1 / sqrt(bc2)).
DEV void adam_elem(float lr, float b1, float b2, float eps, float wd, int decoupled, float& p, float g, float& m,
                   float& v, float step_size, float inv_sqrt_bc2) {
#pragma clang fp contract(off)
  float gr = g;
  if (wd != 0.f) {
    if (decoupled) p *= 1.f - lr * wd;
    else gr += wd * p;
  }
  m = b1 * m + (1.f - b1) * gr;
  v = b2 * v + (1.f - b2) * gr * gr;
  const float denom = sqrtf(v) * inv_sqrt_bc2 + eps;
  p -= step_size * m / denom;
}

DEV void adam_bias_corr(const int* step, float lr, float b1, float b2, float& step_size, float& inv_sqrt_bc2) {
  const int t = step[0];
  const float bc1 = 1.f - powf(b1, (float)t);
  const float bc2 = 1.f - powf(b2, (float)t);
  step_size = lr / bc1;
  inv_sqrt_bc2 = 1.f / sqrtf(bc2);
}

struct AdamArgs {
  float* p;
  const float* g;
  float* m;
  float* v;
  bf16_t* shadow;
  long long n4;
  const int* step;
  float lr, b1, b2, eps, wd;
  int decoupled;
  long long skip_off4, skip_end4;  // float4 range whose rows may be skipped
  int row4;                         // float4s per row in that range
  const unsigned char* touched;     // sticky row flags: nonzero Adam state (nullable)
  const unsigned char* now;         // rows with a valid gradient this step (nullable = all)
  // Disjoint float4 runs of the arena to update ([start4, count4, first virtual index] each,
  // ascending), nullable = all of [0, n4).  Used when the weight-gradient GEMMs already
  // applied Adam to the encoder matrices in their epilogues: one launch covers the rest.
  const long long* runs;
  int nruns;
};

// virtual index -> arena float4 index through the run table (binary search on the prefix)
DEV long long run_index(const long long* runs, int nruns, long long i) {
  int lo = 0, hi = nruns - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (runs[3 * mid + 2] <= i) lo = mid;
    else hi = mid - 1;
  }
  return runs[3 * lo] + (i - runs[3 * lo + 2]);
}

// NT: the moments (and the gradient) are touched once per step -> stream them with
// nontemporal loads/stores so they do not evict the weights / bf16 shadow the next
// forward re-reads from L2 / MALL.
DEV float4 ld_nt(const float4* p) {
  const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  return make_float4(v[0], v[1], v[2], v[3]);
}
DEV void st_nt(float4* p, float4 v) {
  __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4*>(p));
}

// The Adam update of 4 elements (adam_elem each).
DEV void adam_math4(const AdamArgs& a, float (&pp)[4], const float (&gg)[4], float (&mm)[4], float (&vv)[4],
                    float step_size, float inv_sqrt_bc2) {
#pragma unroll
  for (int e = 0; e < 4; ++e)
    adam_elem(a.lr, a.b1, a.b2, a.eps, a.wd, a.decoupled, pp[e], gg[e], mm[e], vv[e], step_size, inv_sqrt_bc2);
}

// One flagged row of a [rows][row4] float4 table starting at float4 base4 (one wave; gradient 0
// unless now[row]).
DEV void adam_row(const AdamArgs& a, long long base4, int row, int row4, int lane, float step_size,
                  float inv_sqrt_bc2) {
  const bool gvalid = a.now == nullptr || a.now[row] != 0;
  for (int c = lane; c < row4; c += 64) {
    const long long i = base4 + (long long)row * row4 + c;
    const float4 p = ld_nt(reinterpret_cast<const float4*>(a.p) + i);
    const float4 g = gvalid ? ld_nt(reinterpret_cast<const float4*>(a.g) + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 m = ld_nt(reinterpret_cast<const float4*>(a.m) + i);
    const float4 v = ld_nt(reinterpret_cast<const float4*>(a.v) + i);
    float pp[4] = {p.x, p.y, p.z, p.w}, gg[4] = {g.x, g.y, g.z, g.w};
    float mm[4] = {m.x, m.y, m.z, m.w}, vv[4] = {v.x, v.y, v.z, v.w};
    adam_math4(a, pp, gg, mm, vv, step_size, inv_sqrt_bc2);
    st_nt(reinterpret_cast<float4*>(a.p) + i, make_float4(pp[0], pp[1], pp[2], pp[3]));
    st_nt(reinterpret_cast<float4*>(a.m) + i, make_float4(mm[0], mm[1], mm[2], mm[3]));
    st_nt(reinterpret_cast<float4*>(a.v) + i, make_float4(vv[0], vv[1], vv[2], vv[3]));
    if (a.shadow) reinterpret_cast<uint2*>(a.shadow)[i] = make_uint2(pack_bf2(pp[0], pp[1]), pack_bf2(pp[2], pp[3]));
  }
}


// One float4 of a flat / run-table Adam (adam_kernel's body; NT: nontemporal g / m / v, NTP: also p).
template <bool NT, bool NTP>
DEV void adam_flat4(const AdamArgs& a, long long vi, float step_size, float inv_sqrt_bc2) {
  const long long i = a.runs ? run_index(a.runs, a.nruns, vi) : vi;
  // Rows never touched since the moments were reset have m = v = g = 0: their
  // Adam update is exactly zero, so skip all their traffic (wd == 0 only).
  bool gvalid = true;
  if (a.touched && i >= a.skip_off4 && i < a.skip_end4) {
    const long long row = (i - a.skip_off4) / a.row4;
    if (!a.touched[row]) return;
    gvalid = a.now == nullptr || a.now[row] != 0;
  }
  float4 p = NTP ? ld_nt(reinterpret_cast<const float4*>(a.p) + i) : reinterpret_cast<float4*>(a.p)[i];
  float4 g, m, v;
  if constexpr (NT) {
    g = gvalid ? ld_nt(reinterpret_cast<const float4*>(a.g) + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    m = ld_nt(reinterpret_cast<const float4*>(a.m) + i);
    v = ld_nt(reinterpret_cast<const float4*>(a.v) + i);
  } else {
    g = gvalid ? reinterpret_cast<const float4*>(a.g)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    m = reinterpret_cast<float4*>(a.m)[i];
    v = reinterpret_cast<float4*>(a.v)[i];
  }
  float pp[4] = {p.x, p.y, p.z, p.w}, gg[4] = {g.x, g.y, g.z, g.w};
  float mm[4] = {m.x, m.y, m.z, m.w}, vv[4] = {v.x, v.y, v.z, v.w};
  adam_math4(a, pp, gg, mm, vv, step_size, inv_sqrt_bc2);
  if constexpr (NTP)
    st_nt(reinterpret_cast<float4*>(a.p) + i, make_float4(pp[0], pp[1], pp[2], pp[3]));
  else
    reinterpret_cast<float4*>(a.p)[i] = make_float4(pp[0], pp[1], pp[2], pp[3]);
  if constexpr (NT) {
    st_nt(reinterpret_cast<float4*>(a.m) + i, make_float4(mm[0], mm[1], mm[2], mm[3]));
    st_nt(reinterpret_cast<float4*>(a.v) + i, make_float4(vv[0], vv[1], vv[2], vv[3]));
  } else {
    reinterpret_cast<float4*>(a.m)[i] = make_float4(mm[0], mm[1], mm[2], mm[3]);
    reinterpret_cast<float4*>(a.v)[i] = make_float4(vv[0], vv[1], vv[2], vv[3]);
  }
  if (a.shadow)
    reinterpret_cast<uint2*>(a.shadow)[i] = make_uint2(pack_bf2(pp[0], pp[1]), pack_bf2(pp[2], pp[3]));
}

// One flagged row of a [rows][192 float4] table (the 768-wide word-embedding rows) with every
// load of the row issued before the first update: one memory round trip per row (adam_row walks
// its three float4 columns one round trip each).  The same arithmetic as adam_row.
DEV void adam_row768(const AdamArgs& a, int row, int lane, float step_size, float inv_sqrt_bc2) {
  constexpr int C = 3;  // 192 float4 / 64 lanes
  const bool gvalid = a.now == nullptr || a.now[row] != 0;
  float4 p[C], g[C], m[C], v[C];
#pragma unroll
  for (int k = 0; k < C; ++k) {
    const long long i = (long long)row * 192 + lane + 64 * k;
    p[k] = ld_nt(reinterpret_cast<const float4*>(a.p) + i);
    g[k] = gvalid ? ld_nt(reinterpret_cast<const float4*>(a.g) + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    m[k] = ld_nt(reinterpret_cast<const float4*>(a.m) + i);
    v[k] = ld_nt(reinterpret_cast<const float4*>(a.v) + i);
  }
#pragma unroll
  for (int k = 0; k < C; ++k) {
    const long long i = (long long)row * 192 + lane + 64 * k;
    float pp[4] = {p[k].x, p[k].y, p[k].z, p[k].w}, gg[4] = {g[k].x, g[k].y, g[k].z, g[k].w};
    float mm[4] = {m[k].x, m[k].y, m[k].z, m[k].w}, vv[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
    adam_math4(a, pp, gg, mm, vv, step_size, inv_sqrt_bc2);
    st_nt(reinterpret_cast<float4*>(a.p) + i, make_float4(pp[0], pp[1], pp[2], pp[3]));
    st_nt(reinterpret_cast<float4*>(a.m) + i, make_float4(mm[0], mm[1], mm[2], mm[3]));
    st_nt(reinterpret_cast<float4*>(a.v) + i, make_float4(vv[0], vv[1], vv[2], vv[3]));
    if (a.shadow) reinterpret_cast<uint2*>(a.shadow)[i] = make_uint2(pack_bf2(pp[0], pp[1]), pack_bf2(pp[2], pp[3]));
  }
}

// The flagged rows among rows [r0, r0 + 16) of a [rows][row4] table (one wave: the 16 flags are
// read at once, then the flagged rows one after another).  16-row chunks spread a run of
// consecutive flagged rows (the frequent WordPiece ids cluster) over many waves.
DEV void adam_rows16(const AdamArgs& a, int r0, int rows, int row4, int lane, float step_size, float inv_sqrt_bc2) {
  const int r = r0 + (lane & 15);
  const bool f = lane < 16 && r < rows && a.touched[r] != 0;
  unsigned long long mask = __ballot(f);
  while (mask) {
    const int bit = __builtin_ctzll(mask);
    mask &= mask - 1;
    if (row4 == 192) adam_row768(a, r0 + bit, lane, step_size, inv_sqrt_bc2);
    else adam_row(a, 0, r0 + bit, row4, lane, step_size, inv_sqrt_bc2);
  }
}
