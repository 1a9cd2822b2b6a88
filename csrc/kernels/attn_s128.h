// S <= 128 attention pieces shared by attention.hip and the fused QKV + attention forward launch
// (gemm.hip gemm_attn_fwd_kernel): fragment layouts, AttnArgs, the varlen / [CLS] helpers, the
// staging loops and the forward body.  Included INSIDE the includer's anonymous namespace (as
// adam_common.h), after common.h.  Reference math: HF DistilBERT MultiHeadSelfAttention, reached
// from client1.py:61 (DistilBertForSequenceClassification.from_pretrained) -- see attention.hip.
#pragma once

constexpr int DH = 64;

// Unified swizzle for [64 rows][64 bf16] tiles (128-byte rows, 8 chunks of 16 B):
// chunk c of row r lives at physical chunk c ^ (r & 6).  Checked against gfx950's
// lane groups (MI355X_MICROARCH.md §LDS) by exhaustive simulation:
//  * ds_read_b128 row reads serve lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... in one
//    LDS cycle each: rows 0-3 and 12-15 read chunk c while rows 4-11 read chunk c+1;
//  * ds_read_b64_tr_b16 reads 8 consecutive rows x 2 adjacent chunks per 32-lane half.
// Both are conflict-free with r & 6.  (Round 1's (r>>1&3)<<1 | (r>>3&1) was conflict-free
// for the tr reads but 2-way on every row read -- it assumed 16 consecutive lanes per
// ds_read_b128 group: 21-27 % LDS bank-conflict cycles in the PMC of both kernels.)
DEV int sw(int r) { return r & 6; }
DEV int tile_off(int r, int c) { return r * 128 + ((c ^ sw(r)) << 4); }

// Stage a [64][64] bf16 tile (row stride ld elements) into LDS; 256 threads.  Rows at or
// beyond `nrows` re-read row nrows-1 (varlen: never read past the sequence / buffer end;
// those rows are masked out of every product).
DEV void stage_tile(char* lds, const bf16_t* src, long ld, int tid, int nrows = 64) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = i * 256 + tid;
    const int r = id >> 3, c = id & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(src + (size_t)min(r, nrows - 1) * ld + c * 8);
    *reinterpret_cast<uint4*>(lds + tile_off(r, c)) = v;
  }
}

// Row-read fragment: rows row0 + (lane&15), columns 32*s + 8*(lane>>4) .. +7.
DEV bf16x8 row_frag(const char* lds, int row0, int s, int lane) {
  const int r = row0 + (lane & 15);
  return *reinterpret_cast<const bf16x8*>(lds + tile_off(r, s * 4 + (lane >> 4)));
}

// Transposed fragment with the permuted k order used for accumulator re-use:
// element j of lane group g = row  32*ks + 16*(j>>2) + 4*g + (j&3), column col0 + (lane&15).
DEV bf16x8 tr_frag(const char* lds, int col0, int ks, int lane) {
  const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
  const int c = (col0 >> 3) + (p >> 1);
  bf16x8 out;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = 32 * ks + 16 * h + 4 * g + q;
    const char* addr = lds + tile_off(r, c) + (p & 1) * 8;
    bf16x4v v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) bf16x4v*)(addr));
    out[4 * h + 0] = v[0];
    out[4 * h + 1] = v[1];
    out[4 * h + 2] = v[2];
    out[4 * h + 3] = v[3];
  }
  return out;
}

// Pack accumulator tiles 2ks, 2ks+1 (4 regs each) into a bf16x8 operand in the
// permuted k order matching tr_frag.
// (v_cvt_pk_bf16_f32: round-to-nearest-even like f2bf for every finite value -- P and dS are finite)
DEV bf16x8 pack_acc(const f32x4& a, const f32x4& b) {
  typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
  const u32x4_t w = {pack_bf2(a[0], a[1]), pack_bf2(a[2], a[3]), pack_bf2(b[0], b[1]), pack_bf2(b[2], b[3])};
  return __builtin_bit_cast(bf16x8, w);
}

DEV bf16x8 load_frag_global(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

struct AttnArgs {
  const bf16_t* qkv;    // [B*S, 3D]
  const float* kbias;   // [B, S] additive key mask (0 / -inf)
  bf16_t* ctx;          // fwd out [B*S, D]
  float* lse;           // [B, H, S]
  const bf16_t* dctx;   // bwd in
  const float* delta;   // [B, H, S]
  bf16_t* dqkv;         // bwd out [B*S, 3D]
  const uint32_t* seed_ptr;
  uint32_t site;
  uint32_t drop_threshold;
  float drop_scale;     // 1/(1-p)
  int B, S, H;
  float scale;          // 1/sqrt(64)
  const int* cu;        // varlen: int32 [B+1] packed sequence starts (nullable = padded [B*S] layout)
  int rows;             // varlen: packed rows of qkv/ctx (rows cu[B] .. rows-1 are bucket filler)
  // S <= 128 kernels with dropout (nullable): the forward leaves its keep bits here, the
  // backward reads them instead of re-hashing (bitwise the same masks).  [B*H][128 q][2] u64,
  // bit k of word (q, kt) = keep(q, key 64 kt + k)
  uint64_t* dmask;
  // S <= 128 kernels: only the first q_live query rows of each sequence are needed (0: all) --
  // the pruned last block needs row 0 ([CLS]) only.  The forward leaves ctx / lse of the other
  // rows unwritten; the backward treats them as rows with no gradient (lse = +inf -> P = 0,
  // delta = 0, dQ = 0 written) -- the caller's dctx is 0 on them.
  int q_live;
  // q_live forward of the pruned last block (nullable): also the compact [CLS] rows its out-proj
  // reads -- cxc[b] = ctx of sequence b's [CLS] row and xc[b] = that row of xres (the block's
  // input, the out-proj residual), for b < B; rows B .. Bp-1 (filler) copy row 0.  An empty packed
  // sequence shares its [CLS] row with the next one: that sequence's blocks write its rows too.
  bf16_t* cxc;
  bf16_t* xc;
  const bf16_t* xres;
  int Bp;
  // its q_live backward with compact [CLS] gradients (nullable): dctx is [Bp, D] (row b = sequence
  // b's [CLS] row; the other rows' dO is 0) and the launch also scatters dresc (the out-proj
  // residual gradient, [Bp, D]) into the full layout dres (row cu[b] = dresc[b], other rows 0;
  // a row shared with empty sequences takes the LAST owner's gradient -- ops/kernels.py
  // scatter_rows2's rule, which this replaces)
  const bf16_t* dresc;
  bf16_t* dres;
  // varlen at S > 128 (attention.hip fd_attn_fwd / fd_attn_bwd, FD_ATTN_SPLIT): the launch pair splits
  // the sequences by length -- the S <= 128 kernels take len <= 128, the 64-row kernels the rest
  int split;
};

// ctx / xres head-h slices of [CLS] row `tok` into compact row b (4 lanes x 4 uint2 = 64 columns;
// xv = the xres slice, loaded once by the caller: the filler fan-out below must not pay a
// dependent load per row)
DEV void cls_compact_row(const AttnArgs& a, int b, int h, int g, const uint2 (&ov)[4], const uint2 (&xv)[4]) {
  const int D = a.H * DH;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int c = h * DH + 16 * dt + 4 * g;
    *reinterpret_cast<uint2*>(a.cxc + (size_t)b * D + c) = ov[dt];
    *reinterpret_cast<uint2*>(a.xc + (size_t)b * D + c) = xv[dt];
  }
}
DEV void cls_xres(const AttnArgs& a, size_t tok, int h, int g, uint2 (&xv)[4]) {
  const int D = a.H * DH;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
    xv[dt] = *reinterpret_cast<const uint2*>(a.xres + tok * D + h * DH + 16 * dt + 4 * g);
}
DEV void cls_compact(const AttnArgs& a, int b, size_t tok, int h, int g, const uint2 (&ov)[4]) {
  uint2 xv[4];
  cls_xres(a, tok, h, g, xv);
  cls_compact_row(a, b, h, g, ov, xv);
  if (a.cu)  // empty sequences before b share this [CLS] row
    for (int b2 = b - 1; b2 >= 0 && a.cu[b2] == (int)tok; --b2) cls_compact_row(a, b2, h, g, ov, xv);
  if (tok == 0)  // the filler rows copy row 0
    for (int i = a.B; i < a.Bp; ++i) cls_compact_row(a, i, h, g, ov, xv);
}

// Varlen: the extra grid slice z == B zeroes head h's columns of the filler rows
// (cu[B] .. rows-1) of `out` (`nsec` 64-wide sections, row stride ld): they are read by
// the next GEMMs and must be finite, and no sequence block ever writes them.
DEV void zero_filler_at(const AttnArgs& a, bf16_t* out, long ld, int nsec, int h, int bx, int gx) {
  const int first = a.cu[a.B];
  const int tid = threadIdx.x;
  for (int r0 = first + bx * 64; r0 < a.rows; r0 += gx * 64) {
    for (int id = tid; id < 64 * nsec * 8; id += 256) {
      const int r = r0 + id / (nsec * 8), c = id % (nsec * 8);
      if (r < a.rows)
        *reinterpret_cast<uint4*>(out + (size_t)r * ld + (size_t)(c >> 3) * (a.H * DH) + h * DH + (c & 7) * 8) =
            make_uint4(0u, 0u, 0u, 0u);
    }
  }
}
DEV void zero_filler(const AttnArgs& a, bf16_t* out, long ld, int nsec, int h) {
  zero_filler_at(a, out, ld, nsec, h, blockIdx.x, gridDim.x);
}

// Sequence b's first packed row and length.  Padded layout: b*S and S (keys masked by kbias).
DEV void seq_span(const AttnArgs& a, int b, int& tok0, int& len) {
  if (a.cu) {
    tok0 = a.cu[b];
    len = a.cu[b + 1] - tok0;
  } else {
    tok0 = b * a.S;
    len = a.S;
  }
}
// Additive key mask: kbias (padded layout) or k < len (varlen).
DEV float key_bias(const AttnArgs& a, int tok0, int len, int k) {
  if (a.cu) return k < len ? 0.f : -INFINITY;
  return a.kbias[tok0 + k];
}

DEV uint32_t site_seed(const AttnArgs& a) { return hash32(a.seed_ptr ? a.seed_ptr[0] : 0u, a.site); }

// Diagnostic build only (FD_HIP_EXTRA_FLAGS=-DFD_ATTN_STAMPS=1): wall-clock stamps (100 MHz) of
// wave 0 of every block at the phase boundaries of the S <= 128 kernels, read back with
// fd_attn_stamps (scripts/attn_stamps.py).  Slot 7: XCC << 32 | HW_ID.  The normal build has none.
#ifndef FD_ATTN_STAMPS
#define FD_ATTN_STAMPS 0
#endif
constexpr int ASTAMP_MAXB = 8192;
#if FD_ATTN_STAMPS
__device__ unsigned long long g_astamps[ASTAMP_MAXB * 8];
DEV int astamp_bid() { return blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z); }
#define ASTAMP(i)                                                                                  \
  do {                                                                                             \
    if (threadIdx.x == 0 && astamp_bid() < ASTAMP_MAXB) g_astamps[astamp_bid() * 8 + (i)] = wall_clock64(); \
  } while (0)
DEV void astamp_hwid() {
  if (threadIdx.x == 0 && astamp_bid() < ASTAMP_MAXB) {
    const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
    const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));
    g_astamps[astamp_bid() * 8 + 7] = ((unsigned long long)(xcc & 0xf) << 32) | hw;
  }
}
#else
#define ASTAMP(i) do {} while (0)
DEV void astamp_hwid() {}
#endif


// Stage rows [0, 64*nt) of a [rows][64]-per-head operand into nt swizzled [64][64]
// images (8 KiB apart); rows >= len re-read row len-1.  NT threads.
template <int NT = 512>
DEV void stage_rows(char* lds, const bf16_t* src, long ld, int tid, int nt, int len) {
#pragma unroll
  for (int i = 0; i < 1024 / NT; ++i) {
    const int id = i * NT + tid;
    const int r = id >> 3, c = id & 7;
    if (r < 64 * nt) {
      const uint4 v = *reinterpret_cast<const uint4*>(src + (size_t)min(r, len - 1) * ld + c * 8);
      *reinterpret_cast<uint4*>(lds + (r >> 6) * 8192 + tile_off(r & 63, c)) = v;
    }
  }
}

// The same staging through write-through-coherent (sc1) buffer loads at element offset off0 of
// the buffer rs covers: the fused QKV + attention launch reads tiles other CUs' blocks of the SAME
// launch wrote with sc1 stores (gemm.hip gemm_attn_fwd_kernel; no kernel boundary in between).
constexpr int ATT_SC1 = 16;  // buffer-op cache policy bit sc1, as gemm.hip LN2_SC1
typedef unsigned int att_u32x4 __attribute__((ext_vector_type(4)));
DEV uint4 ld_sc1_16(__amdgpu_buffer_rsrc_t rs, long elem) {
  const att_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(elem * 2), 0, ATT_SC1);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
template <int NT = 512>
DEV void stage_rows_sc1(char* lds, __amdgpu_buffer_rsrc_t rs, long off0, long ld, int tid, int nt, int len) {
#pragma unroll
  for (int i = 0; i < 1024 / NT; ++i) {
    const int id = i * NT + tid;
    const int r = id >> 3, c = id & 7;
    if (r < 64 * nt) {
      const uint4 v = ld_sc1_16(rs, off0 + (long)min(r, len - 1) * ld + c * 8);
      *reinterpret_cast<uint4*>(lds + (r >> 6) * 8192 + tile_off(r & 63, c)) = v;
    }
  }
}

// Forward, S <= 128: every key of the row at once.  The whole row (<= 128 keys, two 64-key
// tiles) fits one wave's registers, so there is no online-softmax rescale: all score MFMAs issue
// back to back (their K fragments read together), ONE row-max reduction, then exp / dropout and
// all P.V MFMAs -- the earlier tile-by-tile loop paid two dependent cross-lane reductions, the
// rescale and a keep-bit OR-reduction per tile, and the kernel spent 60 % of its wave-cycles
// waiting (PMC, profiles/r3_rejected_register_staging.txt).  Varlen key masks are arithmetic
// (k < len), not an LDS table.  Keep bits go out lane-major: u16 [q / 4][kt * 4 + g][q % 4], bit
// 4 t + r = key 64 kt + 16 t + 4 g + r -- each lane stores its own bits, no cross-lane OR, and the
// backward's key-major phase reads the 4 consecutive query rows of a key word with ONE 8-byte read.
// NW waves per block own query rows [blockIdx.x * 16 NW, + 16 NW): NW = 8 -> one block per
// (sequence, head).  (NW = 4, two blocks per (sequence, head), measured no faster:
// profiles/r4_rejected_ab.txt.)
// The body takes its (sequence b, head h, query block bx) and LDS from the caller: the standalone
// kernel below, or the fused QKV + attention launches (gemm.hip).  MODE: 0 Q / K / V from global
// memory, 1 the same through write-through-coherent sc1 loads, 2 already in LDS as the swizzled
// images K = smem, V = smem + 16 KiB, Q = smem + ATT_FWD_SMEM (written by the caller's projection
// tile; rows past the sequence hold finite values of other rows -- masked keys, unstored queries).
constexpr int ATT_FWD_SMEM = 4 * 8192 + 512;
constexpr int ATT_FWD_SMEM_Q = ATT_FWD_SMEM + 2 * 8192;
template <int NW, int MODE>
DEV void attn_fwd_s128_body(const AttnArgs& a, int b, int h, int bx, char* smem) {
  char* ks = smem;
  char* vs = smem + 2 * 8192;
  float* kb = reinterpret_cast<float*>(smem + 4 * 8192);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int S = a.S, H = a.H, D = H * DH, ld3 = 3 * D;
  ASTAMP(0);
  astamp_hwid();
  if (b == a.B) {
    zero_filler_at(a, a.ctx, D, 1, h, bx, 1);
    if (a.cxc && tid < 4) {  // trailing empty sequences' [CLS] row is the (zeroed) filler row cu[B]
      const int tok = a.cu[a.B];
      const uint2 zero[4] = {make_uint2(0u, 0u), make_uint2(0u, 0u), make_uint2(0u, 0u), make_uint2(0u, 0u)};
      for (int b2 = a.B - 1; b2 >= 0 && a.cu[b2] == tok; --b2) {
        if (tok < a.rows) {
          uint2 xv[4];
          cls_xres(a, (size_t)tok, h, tid, xv);
          cls_compact_row(a, b2, h, tid, zero, xv);
        } else {  // (no filler row: zeros)
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) {
            const size_t c = (size_t)b2 * D + h * DH + 16 * dt + 4 * tid;
            *reinterpret_cast<uint2*>(a.cxc + c) = zero[dt];
            *reinterpret_cast<uint2*>(a.xc + c) = zero[dt];
          }
        }
      }
    }
    return;
  }
  int tok0i, len;
  seq_span(a, b, tok0i, len);
  if (a.split && len > 128) return;  // (block-uniform) the 64-row kernel's sequence
  const int nt = (len + 63) >> 6;
  const size_t tok0 = (size_t)tok0i;
  const int qlen = a.q_live > 0 ? min(len, a.q_live) : len;  // query rows needed
  if (bx * 16 * NW >= qlen) return;  // the whole block past the needed rows
  const int q0 = (bx * NW + w) * 16;
  const int q = q0 + (lane & 15);
  const int qr = min(q, len - 1);
  const bool varlen = a.cu != nullptr;
  bf16x8 qf[2];  // this wave's Q rows, fetched together with the K/V staging loads
  if constexpr (MODE == 2) {
    const char* qs = smem + ATT_FWD_SMEM;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) qf[s2] = row_frag(qs + (q0 >> 6) * 8192, q0 & 63, s2, lane);
  } else if constexpr (MODE == 1) {
    // (the resource from the kernel argument alone: uniform; every per-block part in the offset)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.qkv), 0, 0x7fffffff,
                                                                        0x00020000);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      qf[s2] = __builtin_bit_cast(bf16x8, ld_sc1_16(rs, (long)(tok0 + qr) * ld3 + h * DH + 32 * s2 + 8 * g));
    stage_rows_sc1<64 * NW>(ks, rs, (long)tok0 * ld3 + D + h * DH, ld3, tid, nt, len);
    stage_rows_sc1<64 * NW>(vs, rs, (long)tok0 * ld3 + 2 * D + h * DH, ld3, tid, nt, len);
  } else {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) qf[s2] = load_frag_global(a.qkv + (tok0 + qr) * ld3 + h * DH + 32 * s2 + 8 * g);
    stage_rows<64 * NW>(ks, a.qkv + tok0 * ld3 + D + h * DH, ld3, tid, nt, len);
    stage_rows<64 * NW>(vs, a.qkv + tok0 * ld3 + 2 * D + h * DH, ld3, tid, nt, len);
  }
  // (the softmax runs in log2 units: scores and key biases pre-scaled by log2(e), v_exp_f32 direct)
  if (!varlen && tid < 128) kb[tid] = tid < 64 * nt ? key_bias(a, tok0i, len, tid) * LOG2E : -INFINITY;
  __syncthreads();
  ASTAMP(1);
  if (q0 >= qlen) return;  // no barrier follows
  const uint32_t seed = site_seed(a);
  const bool drop = a.drop_threshold != 0;
  // live 16-key sub-tiles (wave-uniform), bit 4 kt + t: at least one unmasked key.  A sub-tile
  // whose keys are all masked has probabilities exactly 0: its MFMAs and exp / hashes are skipped.
  uint32_t live;
  if (varlen) {
    live = (1u << ((len + 15) >> 4)) - 1u;
  } else {
    const uint64_t vk0 = __ballot(kb[lane] != -INFINITY), vk1 = __ballot(kb[64 + lane] != -INFINITY);
    live = 0u;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      live |= (((vk0 >> (16 * t)) & 0xffffull) != 0 ? 1u : 0u) << t;
      live |= (((vk1 >> (16 * t)) & 0xffffull) != 0 ? 1u : 0u) << (4 + t);
    }
  }
  // ---- scores of every key of the row
  f32x4 sc[2][4];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sc[kt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!((live >> (4 * kt + t)) & 1u)) continue;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) sc[kt][t] = mfma16(row_frag(ks + kt * 8192, 16 * t, s2, lane), qf[s2], sc[kt][t]);
    }
  }
  float mx = -INFINITY;
  const float scale2 = a.scale * LOG2E;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (!((live >> (4 * kt + t)) & 1u)) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = 64 * kt + 16 * t + 4 * g + r;
        const float bias = varlen ? (k < len ? 0.f : -INFINITY) : kb[k];
        sc[kt][t][r] = sc[kt][t][r] * scale2 + bias;
        mx = fmaxf(mx, sc[kt][t][r]);
      }
    }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  const float mref = mx == -INFINITY ? 0.f : mx;
  const uint32_t rowidx = ((uint32_t)(b * H + h) * S + q) * (uint32_t)S;
  float l = 0.f;
  uint32_t kw[2] = {0u, 0u};  // this lane's keep bits per key tile (bit 4 t + r)
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (!((live >> (4 * kt + t)) & 1u)) continue;  // stays 0: exp(-inf) = 0, nothing to hash
      const uint32_t kbits = drop ? drop_keep_bits<4>(seed, rowidx + 64 * kt + 16 * t + 4 * g, a.drop_threshold) : 0xfu;
      if (drop) kw[kt] |= kbits << (4 * t);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = __builtin_amdgcn_exp2f(sc[kt][t][r] - mref);
        l += pv;
        sc[kt][t][r] = (kbits >> r) & 1u ? pv : 0.f;  // (the dropout scale is applied with 1 / l)
      }
    }
  // ---- P . V over every live 32-key half
  f32x4 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (!((live >> (4 * kt + 2 * kk)) & 3u)) continue;
      const bf16x8 pf = pack_acc(sc[kt][2 * kk], sc[kt][2 * kk + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] = mfma16(tr_frag(vs + kt * 8192, 16 * dt, kk, lane), pf, o[dt]);
    }
  if (drop && a.dmask) {
    uint16_t* dm = reinterpret_cast<uint16_t*>(a.dmask) + ((((size_t)b * H + h) * 32 + (q >> 2)) * 8 + g) * 4 + (q & 3);
    dm[0] = (uint16_t)kw[0];
    dm[16] = (uint16_t)kw[1];  // word 4 + g
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  ASTAMP(2);
  if (q >= qlen) return;
  const float inv = (drop ? a.drop_scale : 1.f) / l;
  bf16_t* out = a.ctx + (tok0 + q) * D + h * DH;
  uint2 ov[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    ov[dt] = make_uint2(pack_bf2(o[dt][0] * inv, o[dt][1] * inv), pack_bf2(o[dt][2] * inv, o[dt][3] * inv));
    *reinterpret_cast<uint2*>(out + 16 * dt + 4 * g) = ov[dt];
  }
  if (g == 0) a.lse[((size_t)b * H + h) * S + q] = mref * LN2 + __logf(l);
  if (a.cxc && q == 0) cls_compact(a, b, tok0, h, g, ov);
  ASTAMP(3);
}

// stage_rows in two halves: the loads into registers, then the LDS stores (NT = 512)
DEV void stage_rows_ld(const bf16_t* src, long ld, int tid, int nt, int len, uint4 (&v)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = i * 512 + tid;
    const int r = id >> 3, c = id & 7;
    v[i] = r < 64 * nt ? *reinterpret_cast<const uint4*>(src + (size_t)min(r, len - 1) * ld + c * 8)
                       : make_uint4(0u, 0u, 0u, 0u);
  }
}
DEV void stage_rows_st(char* lds, int tid, int nt, const uint4 (&v)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = i * 512 + tid;
    const int r = id >> 3, c = id & 7;
    if (r < 64 * nt) *reinterpret_cast<uint4*>(lds + (r >> 6) * 8192 + tile_off(r & 63, c)) = v[i];
  }
}

// ---- S <= 128 backward phases (shared by the fused one-block kernel and the two-block split)
// Scores and biases in log2 units: P = exp2(s * scale * log2e + bias2 - lse2).

// Phase 1 for this wave's 16 query rows (lane row q, read row qr = min(q, len - 1)): dQ from the
// K / V images in LDS, the rows' Q / dO fragments, delta dl, lse2 and the forward's keep-bit words
// (mrow_p[kt * 16] = this lane's u16 of key tile kt; null without stored keep bits).
DEV void bwd_dq_rows(const AttnArgs& a, const char* ks, const char* vs, const float* kb, uint64_t vk0,
                     uint64_t vk1, const bf16x8 (&qf)[2], const bf16x8 (&dof)[2], float dl, float lse,
                     const uint16_t* mrow_p, int b, int h, int q, int len, int nt, size_t tok0, int lane) {
  const int g = lane >> 4, S = a.S, H = a.H, D = H * DH, ld3 = 3 * D;
  const bool drop = a.drop_threshold != 0, varlen = a.cu != nullptr;
  const uint32_t seed = site_seed(a);
  const float scale2 = a.scale * LOG2E;
  const uint32_t rowidx = ((uint32_t)(b * H + h) * S + q) * (uint32_t)S;
  f32x4 dq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const uint64_t vk = kt ? vk1 : vk0;
    if (kt >= nt || vk == 0) continue;  // fully masked key tile: dS = 0
    bool tv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) tv[t] = ((vk >> (16 * t)) & 0xffffull) != 0;
    const char* kst = ks + kt * 8192;
    const char* vst = vs + kt * 8192;
    const uint32_t mrow = (drop && mrow_p) ? mrow_p[kt * 16] : 0u;  // this lane's keys 16 t + 4 g + r
    f32x4 sc[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!tv[t]) continue;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        sc[t] = mfma16(row_frag(kst, 16 * t, s2, lane), qf[s2], sc[t]);
        dp[t] = mfma16(row_frag(vst, 16 * t, s2, lane), dof[s2], dp[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (!tv[t]) continue;  // sc[t] = 0 = dS of a fully masked sub-tile
      const uint32_t kw = !drop   ? 0xfu
                          : mrow_p ? (mrow >> (4 * t)) & 0xfu
                                   : drop_keep_bits<4>(seed, rowidx + kt * 64 + 16 * t + 4 * g, a.drop_threshold);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kl = 16 * t + 4 * g + r;
        const float bias = varlen ? (kt * 64 + kl < len ? 0.f : -INFINITY) : kb[kt * 64 + kl];
        const float pv = __builtin_amdgcn_exp2f(sc[t][r] * scale2 + bias - lse);
        float dpv = dp[t][r];
        if (drop) dpv = (kw >> r) & 1u ? dpv * a.drop_scale : 0.f;
        sc[t][r] = pv * (dpv - dl);  // dS
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (!(tv[2 * kk] || tv[2 * kk + 1])) continue;
      const bf16x8 df = pack_acc(sc[2 * kk], sc[2 * kk + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma16(tr_frag(kst, 16 * dt, kk, lane), df, dq[dt]);
    }
  }
  if (q < len) {
    const float sc_out = a.scale;
    bf16_t* out = a.dqkv + (tok0 + q) * ld3 + h * DH;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
      *reinterpret_cast<uint2*>(out + 16 * dt + 4 * g) = make_uint2(
          pack_bf2(dq[dt][0] * sc_out, dq[dt][1] * sc_out), pack_bf2(dq[dt][2] * sc_out, dq[dt][3] * sc_out));
  }
}

// Phase 2 for this wave's 16 keys key0 .. key0 + 15: dK and dV from the Q / dO images in LDS, the
// keys' K / V fragments, lse2 / delta of every query row (LDS) and the keep bits (LDS, mk16).
DEV void bwd_dkv_keys(const AttnArgs& a, const char* qs, const char* os, const float* lse_s, const float* dl_s,
                      const uint16_t* mk16, bool keys_live, const bf16x8 (&kf)[2], const bf16x8 (&vf)[2],
                      float kbias, int b, int h, int key, int len, int nt, int qlen, size_t tok0, int lane) {
  const int g = lane >> 4, S = a.S, H = a.H, D = H * DH, ld3 = 3 * D;
  const bool drop = a.drop_threshold != 0;
  const uint32_t seed = site_seed(a);
  const float scale2 = a.scale * LOG2E;
  const uint32_t headidx = (uint32_t)(b * H + h) * S;
  // this lane's key in the forward's lane-major keep bits: word kt * 4 + g', bit 4 t' + r'
  const int kword = (key >> 6) * 4 + ((key >> 2) & 3), kbit = 4 * ((key >> 4) & 3) + (key & 3);
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    dk[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    if (!keys_live || qt >= nt) continue;
    const char* qst = qs + qt * 8192;
    const char* ost = os + qt * 8192;
    // 16-query sub-tiles past the sequence (varlen) have lse = +inf: P = dS = 0, skipped
    bool tv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) tv[t] = qt * 64 + 16 * t < qlen;
    f32x4 sc[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!tv[t]) continue;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        sc[t] = mfma16(row_frag(qst, 16 * t, s2, lane), kf[s2], sc[t]);  // S[q][key]
        dp[t] = mfma16(row_frag(ost, 16 * t, s2, lane), vf[s2], dp[t]);  // dP[q][key]
      }
    }
    // one 32-query half at a time: P / dS of tiles 2kk, 2kk+1 are packed to bf16 right away
    // (keeps the live set small -> several blocks per CU)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (!(tv[2 * kk] || tv[2 * kk + 1])) continue;
      f32x4 pd[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int t = 2 * kk + u;
        if (!tv[t]) {
          pd[u] = f32x4{0.f, 0.f, 0.f, 0.f};
          continue;  // sc[t] = 0 already
        }
        // the 4 query rows of this lane: one 16-byte LDS read each for their lse and delta
        const float4 lse4 = *reinterpret_cast<const float4*>(lse_s + qt * 64 + 16 * t + 4 * g);
        const float4 dl4 = *reinterpret_cast<const float4*>(dl_s + qt * 64 + 16 * t + 4 * g);
        const float lsev[4] = {lse4.x, lse4.y, lse4.z, lse4.w}, dlv[4] = {dl4.x, dl4.y, dl4.z, dl4.w};
        // the key's words of the 4 query rows: one 8-byte LDS read
        const uint64_t kq = (drop && mk16)
            ? *reinterpret_cast<const uint64_t*>(mk16 + (((qt * 16 + 4 * t + g) * 8 + kword) << 2)) : 0ull;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = qt * 64 + 16 * t + 4 * g + r;
          const float pv = __builtin_amdgcn_exp2f(sc[t][r] * scale2 + kbias - lsev[r]);
          float dpv = dp[t][r], pdv = pv;
          if (drop) {
            const bool keep = mk16 ? ((kq >> (16 * r + kbit)) & 1ull) != 0
                                   : drop_keep(seed, (headidx + ql) * (uint32_t)S + key, a.drop_threshold);
            dpv = keep ? dpv * a.drop_scale : 0.f;
            pdv = keep ? pv : 0.f;  // (the dropout scale is applied to dV once, at the store)
          }
          pd[u][r] = pdv;
          sc[t][r] = pv * (dpv - dlv[r]);  // dS
        }
      }
      const bf16x8 pf = pack_acc(pd[0], pd[1]);
      const bf16x8 sf = pack_acc(sc[2 * kk], sc[2 * kk + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = mfma16(tr_frag(ost, 16 * dt, kk, lane), pf, dv[dt]);
        dk[dt] = mfma16(tr_frag(qst, 16 * dt, kk, lane), sf, dk[dt]);
      }
    }
  }
  if (key >= len) return;
  const float sc_out = a.scale, dv_sc = drop ? a.drop_scale : 1.f;
  bf16_t* outk = a.dqkv + (tok0 + key) * ld3 + D + h * DH;
  bf16_t* outv = a.dqkv + (tok0 + key) * ld3 + 2 * D + h * DH;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    *reinterpret_cast<uint2*>(outk + 16 * dt + 4 * g) = make_uint2(
        pack_bf2(dk[dt][0] * sc_out, dk[dt][1] * sc_out), pack_bf2(dk[dt][2] * sc_out, dk[dt][3] * sc_out));
    *reinterpret_cast<uint2*>(outv + 16 * dt + 4 * g) = make_uint2(
        pack_bf2(dv[dt][0] * dv_sc, dv[dt][1] * dv_sc), pack_bf2(dv[dt][2] * dv_sc, dv[dt][3] * dv_sc));
  }
}

// delta = rowsum(dO * O) of the lane's row from its two 32-wide fragment halves (16 lanes per row)
DEV float row_delta(const bf16x8 (&of)[2], const bf16x8 (&dof)[2]) {
  float dl = 0.f;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int j = 0; j < 8; ++j) dl += bf2f((uint16_t)of[s2][j]) * bf2f((uint16_t)dof[s2][j]);
  dl += __shfl_xor(dl, 16, 64);
  dl += __shfl_xor(dl, 32, 64);
  return dl;
}

// dO tiles of a compact-[CLS] backward (AttnArgs::dresc): row 0 = the sequence's compact row,
// every other row 0 (what stage_rows reads from the scattered layout, clamp included)
template <int NT = 512>
DEV void stage_cls_rows(char* lds, const bf16_t* src, int tid, int nt, int len) {
#pragma unroll
  for (int i = 0; i < 1024 / NT; ++i) {
    const int id = i * NT + tid;
    const int r = id >> 3, c = id & 7;
    if (r < 64 * nt) {
      const uint4 v = min(r, len - 1) == 0 ? *reinterpret_cast<const uint4*>(src + c * 8) : make_uint4(0u, 0u, 0u, 0u);
      *reinterpret_cast<uint4*>(lds + (r >> 6) * 8192 + tile_off(r & 63, c)) = v;
    }
  }
}

// Head h's columns of the sequence's rows of dres: row 0 = dresc[b], the others 0.
template <int NT = 512>
DEV void scatter_cls_rows(const AttnArgs& a, int b, size_t tok0, int len, int h, int tid) {
  const int D = a.H * DH;
  for (int id = tid; id < len * 8; id += NT) {
    const int r = id >> 3, c = id & 7;
    const uint4 v = r == 0 ? *reinterpret_cast<const uint4*>(a.dresc + (size_t)b * D + h * DH + c * 8)
                           : make_uint4(0u, 0u, 0u, 0u);
    *reinterpret_cast<uint4*>(a.dres + (tok0 + r) * D + h * DH + c * 8) = v;
  }
}

// Zero dQ of rows without a gradient (q_live: not among the query rows the loss reaches).
DEV void zero_dq_rows(const AttnArgs& a, int h, int q, int len, size_t tok0, int g) {
  if (q >= len) return;
  bf16_t* out = a.dqkv + (tok0 + q) * (3 * a.H * DH) + h * DH;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) *reinterpret_cast<uint2*>(out + 16 * dt + 4 * g) = make_uint2(0u, 0u);
}

// One block per (sequence, head): phase 1 (waves own 16 query rows: delta, dQ), a barrier, phase 2
// (waves own 16 keys: dK, dV) from the same four LDS images.  (A dQ block beside a dK/dV block per
// (sequence, head) lost its A/B: 23.8 vs 19.3 us per layer, profiles/r4_rejected_ab.txt.)
// MODE 0: dO staged from a.dctx (or the compact [CLS] rows); MODE 2: the caller's proj(tok0, len)
// computes the dO image itself (gemm.hip attn_bwd_proj_kernel: the out-projection's dX tile), using
// smem[0, 48 KiB) -- the Q / K / V image region -- as its operand ring: Q / K / V are loaded into
// registers before it runs and stored to LDS after it returns (it ends with a workgroup barrier).
constexpr int ATT_BWD_SMEM = 8 * 8192 + 3 * 512 + 2048;
struct NoProj {
  DEV void operator()(int, int) const {}
};
template <int MODE, class ProjFn>
DEV void attn_bwd_s128_body(const AttnArgs& a, int b, int h, char* smem, const ProjFn& proj) {
  char* qs = smem;
  char* ks = smem + 2 * 8192;
  char* vs = smem + 4 * 8192;
  char* os = smem + 6 * 8192;  // dO
  float* kb = reinterpret_cast<float*>(smem + 8 * 8192);
  float* lse_s = kb + 128;
  float* dl_s = lse_s + 128;
  uint64_t* mk_s = reinterpret_cast<uint64_t*>(smem + 8 * 8192 + 3 * 512);  // the forward's keep bits
  const uint16_t* mk16 = reinterpret_cast<const uint16_t*>(mk_s);  // [q / 4][kt * 4 + g][q % 4], bit 4 t + r

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int S = a.S, H = a.H, D = H * DH, ld3 = 3 * D;
  ASTAMP(0);
  astamp_hwid();
  if (b == a.B) {
    zero_filler_at(a, a.dqkv, ld3, 3, h, 0, 1);
    if (a.dres) {
      zero_filler_at(a, a.dres, D, 1, h, 0, 1);
      const int tok = a.cu[a.B];  // trailing empty sequences: the last one's gradient on row cu[B]
      if (a.B > 0 && a.cu[a.B - 1] == tok && tok < a.rows) {
        __syncthreads();
        if (tid < 8)
          *reinterpret_cast<uint4*>(a.dres + (size_t)tok * D + h * DH + tid * 8) =
              *reinterpret_cast<const uint4*>(a.dresc + (size_t)(a.B - 1) * D + h * DH + tid * 8);
      }
    }
    return;
  }
  int tok0i, len;
  seq_span(a, b, tok0i, len);
  const int nt = (len + 63) >> 6;
  const int qlen = a.q_live > 0 ? min(len, a.q_live) : len;  // query rows with a gradient
  // an empty sequence (varlen) owns no rows: nothing to write, and its clamped row len - 1 = -1
  // must not be read (a leading empty sequence would read before the tensors)
  if (len == 0 || (a.split && len > 128)) return;  // (split: the 64-row kernels' sequence)
  const size_t tok0 = (size_t)tok0i;
  const size_t st0 = ((size_t)b * H + h) * S;
  // phase 1's O rows (for delta) are fetched together with the staging loads: no second
  // dependent global round trip after the barrier
  const int q0 = w * 16;
  bf16x8 of[2];
  {
    const int qr = min(q0 + (lane & 15), len - 1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) of[s2] = load_frag_global(a.ctx + (tok0 + qr) * D + h * DH + 32 * s2 + 8 * g);
  }
  if constexpr (MODE == 2) {
    uint4 qv[2], kv[2], vv[2];  // in flight across the dO projection's K loop
    stage_rows_ld(a.qkv + tok0 * ld3 + h * DH, ld3, tid, nt, len, qv);
    stage_rows_ld(a.qkv + tok0 * ld3 + D + h * DH, ld3, tid, nt, len, kv);
    stage_rows_ld(a.qkv + tok0 * ld3 + 2 * D + h * DH, ld3, tid, nt, len, vv);
    proj(tok0i, len);  // the dO image (os); its ring in [qs, os) is free again when it returns
    stage_rows_st(qs, tid, nt, qv);
    stage_rows_st(ks, tid, nt, kv);
    stage_rows_st(vs, tid, nt, vv);
  } else {
    stage_rows(qs, a.qkv + tok0 * ld3 + h * DH, ld3, tid, nt, len);
    stage_rows(ks, a.qkv + tok0 * ld3 + D + h * DH, ld3, tid, nt, len);
    stage_rows(vs, a.qkv + tok0 * ld3 + 2 * D + h * DH, ld3, tid, nt, len);
    if (a.dres)
      stage_cls_rows(os, a.dctx + (size_t)b * D + h * DH, tid, nt, len);
    else
      stage_rows(os, a.dctx + tok0 * D + h * DH, D, tid, nt, len);
  }
  if (tid < 128) {
    kb[tid] = tid < 64 * nt ? key_bias(a, tok0i, len, tid) * LOG2E : -INFINITY;
    // query rows past the sequence: lse = +inf makes their P (and dS) exactly 0
    lse_s[tid] = tid < qlen ? a.lse[st0 + tid] * LOG2E : INFINITY;
    dl_s[tid] = 0.f;
  }
  // the forward's keep bits (rows the forward did not write are past the sequence: P = 0 there)
  const bool mk = a.drop_threshold != 0 && a.dmask != nullptr;
  if (mk && tid < 256) mk_s[tid] = a.dmask[((size_t)b * H + h) * 256 + tid];
  // (after the staging loads are issued: wave 0's [CLS] row store waits for its load)
  if (a.dres) scatter_cls_rows(a, b, tok0, len, h, tid);
  __syncthreads();
  ASTAMP(1);
  // unmasked-key bits of the two 64-key tiles (see attn_fwd_s128_kernel): 16-key sub-tiles
  // with every key masked have P = dS = 0 exactly and are skipped in both phases
  const uint64_t vk0 = __ballot(kb[lane] != -INFINITY);
  const uint64_t vk1 = __ballot(kb[64 + lane] != -INFINITY);

  // ---- phase 1: dQ and delta; wave w owns queries 16w .. 16w+15
  if (q0 >= qlen && q0 < len) zero_dq_rows(a, h, q0 + (lane & 15), len, tok0, g);
  if (q0 < qlen) {
    const int q = q0 + (lane & 15);
    const int qr = min(q, len - 1);
    bf16x8 qf[2], dof[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      qf[s2] = row_frag(qs + (q0 >> 6) * 8192, q0 & 63, s2, lane);
      dof[s2] = row_frag(os + (q0 >> 6) * 8192, q0 & 63, s2, lane);
    }
    float dl = row_delta(of, dof);
    if (q >= qlen) dl = 0.f;  // (q_live: this row's O was never written -- it has no gradient)
    if (g == 0 && q < len) dl_s[q] = dl;
    const uint16_t* mrow_p = mk ? mk16 + ((qr >> 2) * 8 + g) * 4 + (qr & 3) : nullptr;
    bwd_dq_rows(a, ks, vs, kb, vk0, vk1, qf, dof, dl, lse_s[qr], mrow_p, b, h, q, len,
                nt, tok0, lane);
  }
  ASTAMP(2);
  __syncthreads();  // delta of every query row is in LDS
  ASTAMP(3);

  // ---- phase 2: dK and dV; wave w owns keys 16w .. 16w+15
  const int key0 = w * 16;
  if (key0 >= len) return;
  bf16x8 kf[2], vf[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    kf[s2] = row_frag(ks + (key0 >> 6) * 8192, key0 & 63, s2, lane);
    vf[s2] = row_frag(vs + (key0 >> 6) * 8192, key0 & 63, s2, lane);
  }
  // this wave's 16 keys all masked (padded layout): P and dS columns are 0, dK = dV = 0
  const bool keys_live = (((key0 < 64 ? vk0 >> key0 : vk1 >> (key0 - 64))) & 0xffffull) != 0;
  const int key = key0 + (lane & 15);
  bwd_dkv_keys(a, qs, os, lse_s, dl_s, mk ? mk16 : nullptr, keys_live, kf, vf, kb[key], b, h, key, len, nt, qlen,
               tok0, lane);
  ASTAMP(4);
}
