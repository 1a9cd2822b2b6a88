// bf16 MFMA GEMM with fused epilogues for the DistilBERT projections (gfx950).
//
// C[m][n] = sum_k A(m,k) * B(k,n), fp32 accumulate on v_mfma_f32_16x16x32_bf16.
//   A_KMAJ: A(m,k) = A[m*lda + k]   else A(m,k) = A[k*lda + m]
//   B_KMAJ: B(k,n) = B[n*ldb + k]   else B(k,n) = B[k*ldb + n]
// The three training GEMMs of every nn.Linear (reference: the q/k/v/out_lin,
// ffn.lin1/lin2 projections reached from client1.py:61 via HF DistilBERT):
//   forward  y  = x W^T + b     -> A_KMAJ, B_KMAJ   ("NT")
//   backward dx = dy W          -> A_KMAJ, !B_KMAJ  ("NN")
//   backward dW = dy^T x        -> !A_KMAJ, !B_KMAJ ("TN", split-K fp32 slabs)
//
// Design (MI355X-first, cdna_hip_programming.md §5, "Pipelining across barriers"):
//  * One template over (BM, BN, waves WMxWN, LDS ring depth S); the host picks a
//    measured configuration per shape (cfg table below) so the grid is one
//    full round of 256 CUs wherever the shape allows.
//  * Operand tiles go HBM/L2 -> LDS with global_load_lds_dwordx4 (LDS-DMA, no
//    VGPR round trip) into an S-deep ring.  Per K tile: counted vmcnt that
//    leaves the S-2 younger tiles in flight, ONE raw s_barrier, then the DMA of
//    tile kt+S-1 into the slot everyone just finished reading.
//  * Both 32-deep fragment sets of a K tile are read up front, so the second
//    set's ds_reads overlap the first set's MFMAs.
//  * The DMA writes LDS lane-linearly, so bank-conflict swizzles are applied on
//    the per-lane SOURCE address and undone on the read (rule 21):
//    K-major images [rows][64] use chunk ^= (row>>1)&7 (conflict-free
//    ds_read_b128 fragments); MN-major images are [64 k][64|128 mn] sub-images
//    read with the transposing ds_read_b64_tr_b16 (T10), chunk ^= fk(k).
//  * Operands are swapped inside the MFMA (D = B^T A^T = C^T) so every lane owns
//    4 consecutive output columns.  The epilogue parks the tile in LDS and the
//    whole block writes contiguous 16-byte row chunks (the per-lane 16-row x
//    32-byte store pattern is store-issue bound).
//  * XCD-aware bijective block remap (T1) + group-M tile walk sized to the L2.
#include "common.h"
#include "adam_epi.h"

#include <cstdlib>
#include <cstring>

namespace {

#include "adam_common.h"
#include "attn_s128.h"

enum Epi : int {
  EPI_BF16 = 0,       // C(bf16) = acc
  EPI_BIAS = 1,       // C(bf16) = acc + bias[n]
  EPI_BIAS_GELU = 2,  // aux(bf16) = acc + bias[n];  C(bf16) = gelu(aux)
  EPI_GELU_BWD = 3,   // C(bf16) = acc * gelu'(aux[m][n])
  EPI_ADD = 4,        // C(bf16) = acc + res[m][n]
  EPI_F32 = 5,        // C(fp32 slab z) = acc
  EPI_LN = 6,         // C(bf16) = LN(dropout(acc + bias) + res)    (p.ln; gemm_ln_kernel only)
  EPI_LN_BWD = 7,     // C(bf16) = LN backward of dy = acc + res    (p.ln; gemm_ln_kernel only)
  EPI_LN2 = 8,        // EPI_LN / EPI_LN_BWD of a 128 x 64 tile from the two K halves of a 128 x 128
  EPI_LN2_BWD = 9,    //   product tile (gemm_ln2_kernel only; p.ln2_half = which half this block runs)
};

struct GemmParams {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  int M, N, K;
  int lda, ldb, ldc;
  const float* bias;
  bf16_t* aux;
  int ldaux;
  const bf16_t* res;
  int ldres;
  int k_split;           // K elements per split (multiple of 64)
  long long slab_stride; // elements between fp32 slabs
  int group_m;           // tile-walk group height (L2 working-set control)
  int diag;              // FD_GEMM_DIAG bits (profiling only): 1 no in-loop DMA, 4 no stores,
                         // 128 LN epilogue operands loaded after the K loop (no ln_dma A/B)
  // EPI_F32 destinations (weight gradients).  out == nullptr: slab mode (slab z of C, reduced
  // by splitk_reduce_kernel).  Otherwise one K split: the tile goes straight to the final [M][N]
  // fp32 gradient out (+= out if accumulate).
  float* out;
  int accumulate;
  FdAdamEpi adam;        // adam.p != nullptr: apply Adam to the finished tile instead of storing it
  // EPI_GELU_BWD / EPI_ADD with a staged fp32 tile: column sums of the stored output per M
  // tile, [ceil(M / BM)][N] fp32 (the producer-bias gradient, e.g. FFN lin1's bias)
  float* colsum;
  // EPI_GELU_BWD: also write gelu(aux) here (ld = ldaux; nullable).  The backward re-creates
  // the FFN activation g = gelu(u) next to its consumer (lin2's weight gradient) instead of
  // the forward keeping it: bitwise the forward's values (same bf16 u, same gelu_erf).
  bf16_t* aux_out;
  FdLnEpi ln;            // EPI_LN / EPI_LN_BWD (adam_epi.h)
  // EPI_F32, nullable: acol[m] (+= when accumulate) = sum over the K range of A[k][m], written by
  // the tiles with tn == 0 (FdDwProb::bias)
  float* acol;
  // with the fused Adam (adam.p) and these set: the finished acol[m] is not stored -- Adam (adam_elem,
  // hyper-parameters of `adam`) updates the bias's master / moments / bf16 shadow at that element
  float* acol_p;
  float* acol_m;
  float* acol_v;
  uint16_t* acol_sh;
  int ln2_half;          // EPI_LN2*: this block's K half and the 64-column half of the tile it finishes
};

constexpr int BKT = 64;
constexpr int LDS_MAX = 163840;

// Diagnostic build only (FD_HIP_EXTRA_FLAGS=-DFD_GEMM_STAMPS=1): per-block wall-clock stamps
// (100 MHz) at the phase boundaries of the one-round GEMMs, read back with fd_gemm_stamps
// (scripts/gemm_stamps.py).  Slot 7 holds the hardware id (XCC << 16 | HW_ID).  Nothing of the
// normal build executes or reads them.
#ifndef FD_GEMM_STAMPS
#define FD_GEMM_STAMPS 0
#endif
constexpr int STAMP_MAXB = 2048;
#if FD_GEMM_STAMPS
__device__ unsigned long long g_stamps[STAMP_MAXB * 8];
DEV int stamp_bid() { return blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z); }
#define FD_STAMP(i)                                                                                \
  do {                                                                                             \
    if (threadIdx.x == 0 && stamp_bid() < STAMP_MAXB) g_stamps[stamp_bid() * 8 + (i)] = wall_clock64(); \
  } while (0)
DEV void stamp_hwid() {
  if (threadIdx.x == 0 && stamp_bid() < STAMP_MAXB) {
    const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID
    g_stamps[stamp_bid() * 8 + 7] = ((unsigned long long)(xcc & 0xf) << 32) | hw;
  }
}
#else
#define FD_STAMP(i) do {} while (0)
DEV void stamp_hwid() {}
#endif

// Logical tile id -> (tm, tn).  After the XCD remap each XCD owns a contiguous
// range of logical ids; walking them in groups of `gm` M-tiles x all N-tiles
// means the blocks resident on one XCD share gm A-panels and a few B-panels.
DEV void tile_coords(int lid, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  const int per_group = gm * tiles_n;
  const int group = lid / per_group;
  const int first_m = group * gm;
  const int rows = min(gm, tiles_m - first_m);
  const int in_group = lid - group * per_group;
  tm = first_m + in_group % rows;
  tn = in_group / rows;
}

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

// One 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4): 1 KiB to the wave-uniform LDS address
// `lds`, each lane from its own `src`.  FD_GLDS_ASM (default): issued from inline asm, so hipcc
// does not track it -- the ring's counted s_waitcnt vmcnt (wait_tiles) is the only wait.  With the
// builtin, hipcc cannot tell the DMA's LDS write apart from the transposing ds_read_b64_tr_b16
// fragment reads of MN-major operands and waits vmcnt(0) right after every K tile's DMA issue
// (measured in the .s of every TN weight-gradient kernel): the next tile's DMA latency then sits
// inside the K loop instead of behind the current tile's MFMAs.  Every path drains the ring
// (vmcnt(0)) before the epilogue reuses the LDS, which __syncthreads() alone would not do.
#ifndef FD_GLDS_ASM
#define FD_GLDS_ASM 1
#endif
DEV void glds16(const void* src, char* lds) {
#if FD_GLDS_ASM
  const uint32_t dst = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(lds_void*)lds);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
#else
  __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds, 16, 0, 0);
#endif
}

// Swizzle of 16-byte chunks for an MN-major ([k][mn]) sub-image of width W.
template <int W>
DEV int fk(int k) {
  if constexpr (W == 128) return ((k & 3) | ((k >> 1) & 4)) << 1;
  else return (((k >> 1) & 1) | ((k >> 2) & 2)) << 1;
}

// K-major chunk swizzle for 128-byte rows: 16 consecutive rows reading the same
// logical chunk land on 16 distinct 16-byte bank slots.
DEV int ksw(int r) { return (r >> 1) & 7; }

// BK: K depth of one ring slot -- 64 (two 32-deep MFMA k-steps), or 32 for MN-major operands
// (half the bytes per slot: twice the slots in flight for the same LDS; the all-layer dW launch
// with 4 / 5 such slots lost its A/B, profiles/r4_rejected_ab.txt, and is not instantiated).
template <int ROWS, bool KMAJ, int NWAVES, int BK = BKT>
struct Operand {
  static_assert(BK == BKT || (!KMAJ && BK == 32), "32-deep slots: MN-major images only");
  static constexpr int BYTES = ROWS * BK * 2;               // one LDS slot
  static constexpr int PER_WAVE = BYTES / 1024 / NWAVES;   // 1 KiB DMA pieces per wave per tile
  // MN-major: [BK][SUB] sub-images stacked along mn
  static constexpr int SUB = (ROWS % 128 == 0) ? 128 : 64;
  static constexpr int SUB_BYTES = BK * SUB * 2;
  static constexpr int SUB_CH = SUB / 8;

  // LDS-DMA of the K tile starting at k0.  K-major rows beyond `lim` are clamped
  // (their products land in output rows that are never stored).  Scalar tile
  // base + 32-bit per-lane byte offset (loop-invariant, one VGPR per piece).
  DEV static void stage(const bf16_t* base, int ld, int row0, int k0, int lim, char* lds, int wid, int lane) {
    const char* sbase = reinterpret_cast<const char*>(KMAJ ? base + k0 : base + (size_t)k0 * ld + row0);
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int piece = wid * PER_WAVE + i;
      const int pos = piece * 64 + lane;  // physical 16-byte chunk of the slot
      uint32_t off;
      if constexpr (KMAJ) {
        const int r = pos >> 3, c = (pos & 7) ^ ksw(r);
        const int gr = min(row0 + r, lim - 1);
        off = (uint32_t)(gr * ld + c * 8) * 2u;
      } else {
        const int sub = pos / (SUB_BYTES / 16), lp = pos % (SUB_BYTES / 16);
        const int k = lp / SUB_CH, c = (lp % SUB_CH) ^ fk<SUB>(k);
        off = (uint32_t)(k * ld + sub * SUB + c * 8) * 2u;
      }
      glds16(sbase + off, lds + piece * 1024);
    }
  }


  // MFMA fragment for rows [row0, row0+16) and k-step s (32 deep).
  DEV static bf16x8 frag(const char* lds, int row0, int s, int lane) {
    if constexpr (KMAJ) {
      const int row = row0 + (lane & 15);
      const int c = s * 4 + (lane >> 4);
      return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((c ^ ksw(row)) << 4));
    } else {
      const char* img = lds + (row0 / SUB) * SUB_BYTES;
      const int r0 = row0 % SUB;
      const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
      const int c = (r0 >> 3) + (p >> 1);
      bf16x8 out;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = s * 32 + 8 * g + 4 * h + q;
        const char* addr = img + k * (SUB * 2) + ((c ^ fk<SUB>(k)) << 4) + (p & 1) * 8;
        bf16x4v v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) bf16x4v*)(addr));
        out[4 * h + 0] = v[0];
        out[4 * h + 1] = v[1];
        out[4 * h + 2] = v[2];
        out[4 * h + 3] = v[3];
      }
      return out;
    }
  }
};

constexpr uint32_t LN2_SC1 = 16;  // buffer-op cache policy: sc1 (write-through / L1 bypass)
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- epilogue
// Each wave parks its accumulators in LDS (bias applied; bf16, or fp32 when the
// finishing math needs per-element operands and the fp32 tile fits), then the
// block writes full contiguous rows with 16-byte stores.  Row pitch = payload
// + 16 B: the 16-row ds_write groups land on distinct banks for BN in
// {64, 96, 128, 192, 256}.
template <int EPI, int BM, int BN>
struct EpiTraits {
  static constexpr bool ELEM = (EPI == EPI_ADD || EPI == EPI_GELU_BWD);
  static constexpr bool LN2 = (EPI == EPI_LN2 || EPI == EPI_LN2_BWD);
  static constexpr bool LN = (EPI == EPI_LN || EPI == EPI_LN_BWD || LN2);
  // fp32 weight-gradient tiles too large to stage in LDS (256 x 192, 256 x 256) are finished
  // straight from the accumulators (direct_f32_epilogue): 16-byte stores per lane
  static constexpr bool DIRECT = EPI == EPI_F32 && BM * (BN * 4 + 16) > LDS_MAX;
  static constexpr bool F32S = (EPI == EPI_F32 && !DIRECT) || ((ELEM || LN) && BM * (BN * 4 + 16) <= LDS_MAX);
  static constexpr int ES = F32S ? 4 : 2;
  static constexpr int BYTES = DIRECT ? 0 : BM * (BN * ES + 16);
};

DEV float4 ld_nt4(const float* p) {
  const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  return make_float4(v[0], v[1], v[2], v[3]);
}
DEV void st_nt4(float* p, float4 v) {
  __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4*>(p));
}

// Adam on 4 consecutive elements of a finished gradient tile: adam_elem (adam_common.h), as in
// adam_kernel (head_optim.hip), so a fused step matches the unfused one bitwise.
DEV float4 adam_epi4(const FdAdamEpi& a, size_t i, float4 g4, float step_size, float inv_sqrt_bc2) {
  const float4 p4 = ld_nt4(a.p + i), m4 = ld_nt4(a.m + i), v4 = ld_nt4(a.v + i);
  float pp[4] = {p4.x, p4.y, p4.z, p4.w}, gg[4] = {g4.x, g4.y, g4.z, g4.w};
  float mm[4] = {m4.x, m4.y, m4.z, m4.w}, vv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
  for (int e = 0; e < 4; ++e)
    adam_elem(a.lr, a.b1, a.b2, a.eps, a.wd, a.decoupled, pp[e], gg[e], mm[e], vv[e], step_size, inv_sqrt_bc2);
  st_nt4(a.p + i, make_float4(pp[0], pp[1], pp[2], pp[3]));
  st_nt4(a.m + i, make_float4(mm[0], mm[1], mm[2], mm[3]));
  st_nt4(a.v + i, make_float4(vv[0], vv[1], vv[2], vv[3]));
  if (a.sh) *reinterpret_cast<uint2*>(a.sh + i) = make_uint2(pack_bf2(pp[0], pp[1]), pack_bf2(pp[2], pp[3]));
  return make_float4(pp[0], pp[1], pp[2], pp[3]);
}

// Weight-gradient (fp32) epilogue; see GemmParams::out for the two modes.
template <int BM, int BN, int NT>
DEV void f32_epilogue(const GemmParams& p, const char* smem, int ldc_lds, int m0, int n0, int tid) {
  constexpr int CPR = BN / 4;  // 4 fp32 per chunk
  if (p.out == nullptr) {      // legacy: slab z, reduced by a separate launch
    float* C = reinterpret_cast<float*>(p.C) + (size_t)blockIdx.z * p.slab_stride;
#pragma unroll 4
    for (int id = tid; id < BM * CPR; id += NT) {
      const int r = id / CPR, cc = id - r * CPR;
      const int m = m0 + r;
      if (m >= p.M) break;
      *reinterpret_cast<float4*>(C + (size_t)m * p.ldc + n0 + cc * 4) =
          *reinterpret_cast<const float4*>(smem + r * ldc_lds + cc * 16);
    }
    return;
  }
  const bool adam = p.adam.p != nullptr;
  float step_size = 0.f, inv_sqrt_bc2 = 0.f;
  if (adam) {
    const int t = p.adam.step[0];
    const float bc1 = 1.f - powf(p.adam.b1, (float)t);
    const float bc2 = 1.f - powf(p.adam.b2, (float)t);
    step_size = p.adam.lr / bc1;
    inv_sqrt_bc2 = 1.f / sqrtf(bc2);
  }
#pragma unroll 2
  for (int id = tid; id < BM * CPR; id += NT) {
    const int r = id / CPR, cc = id - r * CPR;
    const int m = m0 + r;
    if (m >= p.M) break;
    const size_t i = (size_t)m * p.ldc + n0 + cc * 4;
    float4 g = *reinterpret_cast<const float4*>(smem + r * ldc_lds + cc * 16);
    if (p.accumulate) {
      const float4 o = *reinterpret_cast<const float4*>(p.out + i);
      g.x += o.x; g.y += o.y; g.z += o.z; g.w += o.w;
    }
    if (adam) {
      adam_epi4(p.adam, i, g, step_size, inv_sqrt_bc2);
    } else {
      *reinterpret_cast<float4*>(p.out + i) = g;
    }
  }
}

// aux_out[m][n..n+3] = gelu(aux[m][n..n+3]) from the 4 bf16 pre-activations already loaded
DEV void gelu_remat(const GemmParams& p, int m, int n, const uint2& u) {
  *reinterpret_cast<uint2*>(p.aux_out + (size_t)m * p.ldaux + n) =
      make_uint2(pack_bf2(gelu_erf(lo_bf(u.x)), gelu_erf(hi_bf(u.x))),
                 pack_bf2(gelu_erf(lo_bf(u.y)), gelu_erf(hi_bf(u.y))));
}

// Next-launch weight prefetch (FdLnEpi::pf, cold operands: profiles/r4_cold_operands.txt -- a QKV
// forward whose weight comes from HBM is ~4 us slower).  Issued just before the row-statistics
// poll: every block loads one dword per 64 bytes of its 1/grid slice of pf (at most PF_N per
// thread), which fills MALL and this XCD's L2 for the next launch.  vmcnt retires loads in order,
// so the first poll also waits for these -- the poll waits ~1.7 us for the slowest tile of the row
// block anyway.  The values are dead: an empty asm at the end of the epilogue consumes them.
constexpr int PF_N = 2;
struct PfRegs {
  uint32_t v[PF_N];
};
template <int NT>
DEV PfRegs pf_issue(const FdLnEpi& L, int tid) {
  PfRegs r;
#pragma unroll
  for (int k = 0; k < PF_N; ++k) r.v[k] = 0u;
  if (L.pf == nullptr) return r;  // (kernel argument: uniform)
  const long long lines = L.pf_bytes >> 6, nb = gridDim.x * gridDim.y;
  const long long per = (lines + nb - 1) / nb;
  const long long c0 = (long long)(blockIdx.y * gridDim.x + blockIdx.x) * per;
  const long long c1 = c0 + per < lines ? c0 + per : lines;
#pragma unroll
  for (int k = 0; k < PF_N; ++k) {
    const long long c = c0 + k * NT + tid;
    if (c < c1) r.v[k] = *reinterpret_cast<const uint32_t*>(L.pf + (c << 6));  // (cached: that is the point)
  }
  return r;
}
DEV void pf_consume(const PfRegs& r) {
#pragma unroll
  for (int k = 0; k < PF_N; ++k) asm volatile("" ::"v"(r.v[k]));
}

template <int BM, int BN, int TM, int TN, int EPI, int NT, int NPRE, bool WT = false>
DEV void staged_epilogue_out(const GemmParams& p, char* smem, int m0, int n0, int tid, const uint4 (&pre)[NPRE]);

// WT: the bf16 tile goes out with write-through (sc1) stores that every thread drains before
// returning (the fused QKV + attention launch: blocks of the same launch on other XCDs read it)
template <int BM, int BN, int TM, int TN, int EPI, int NT, bool WT = false>
DEV void staged_epilogue(const GemmParams& p, const f32x4 (&acc)[TM / 16][TN / 16], char* smem, int m0, int n0,
                         int wr, int wc, int lane, int tid) {
  using TR = EpiTraits<EPI, BM, BN>;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int LDC = BN * TR::ES + 16;
  // staged element epilogues: this thread's aux / residual chunks (16 B each) are all loaded up
  // front, in flight while the tile is parked -- in the chunk loop below each load would wait
  // for the previous chunk's store (they may alias), one chunk per thread in flight
  constexpr int CPR8 = BN / 8, NCH = BM * CPR8 / NT;
  constexpr bool PRE = TR::ELEM && TR::F32S && (BM * CPR8) % NT == 0 && NCH <= 8;
  // (1.581 vs 1.590 ms/step, profiles/r5_ab_elem_epilogue_prefetch.txt)
  uint4 pre[PRE ? NCH : 1];
  if constexpr (PRE) {
    const bf16_t* src = EPI == EPI_GELU_BWD ? p.aux : p.res;
    const int lds = EPI == EPI_GELU_BWD ? p.ldaux : p.ldres;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int id = tid + k * NT, r = id / CPR8, cc = id - r * CPR8;
      pre[k] = *reinterpret_cast<const uint4*>(src + (size_t)min(m0 + r, p.M - 1) * lds + n0 + cc * 8);
    }
  }
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int r = wr * TM + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int c = wc * TN + j * 16 + 4 * (lane >> 4);
      float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
      if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
        const float4 b = *reinterpret_cast<const float4*>(p.bias + n0 + c);
        v0 += b.x; v1 += b.y; v2 += b.z; v3 += b.w;
      }
      if constexpr (TR::ELEM && !TR::F32S) {  // big tile: finish in registers (scattered 8-byte loads)
        const int m = min(m0 + r, p.M - 1), n = n0 + c;
        if constexpr (EPI == EPI_GELU_BWD) {
          const uint2 u = *reinterpret_cast<const uint2*>(p.aux + (size_t)m * p.ldaux + n);
          v0 *= gelu_erf_grad(lo_bf(u.x)); v1 *= gelu_erf_grad(hi_bf(u.x));
          v2 *= gelu_erf_grad(lo_bf(u.y)); v3 *= gelu_erf_grad(hi_bf(u.y));
          if (p.aux_out && m0 + r < p.M) gelu_remat(p, m, n, u);
        } else {
          const uint2 r2 = *reinterpret_cast<const uint2*>(p.res + (size_t)m * p.ldres + n);
          v0 += lo_bf(r2.x); v1 += hi_bf(r2.x); v2 += lo_bf(r2.y); v3 += hi_bf(r2.y);
        }
      }
      if constexpr (TR::F32S) {
        *reinterpret_cast<float4*>(smem + r * LDC + c * 4) = make_float4(v0, v1, v2, v3);
      } else {
        *reinterpret_cast<uint2*>(smem + r * LDC + c * 2) = make_uint2(pack_bf2(v0, v1), pack_bf2(v2, v3));
      }
    }
  }
  __syncthreads();
  if (p.diag & 4) return;
  if constexpr (EPI == EPI_F32) {  // (weight gradients: no next-launch prefetch)
    staged_epilogue_out<BM, BN, TM, TN, EPI, NT>(p, smem, m0, n0, tid, pre);
  } else {
    // the next launch's weight (p.ln.pf, fd_gemm_pf): issued after every load this epilogue waits for
    const PfRegs pfr = pf_issue<NT>(p.ln, tid);
    staged_epilogue_out<BM, BN, TM, TN, EPI, NT, PRE ? NCH : 1, WT>(p, smem, m0, n0, tid, pre);
    pf_consume(pfr);
  }
}

template <int BM, int BN, int TM, int TN, int EPI, int NT, int NPRE, bool WT>
DEV void staged_epilogue_out(const GemmParams& p, char* smem, int m0, int n0, int tid, const uint4 (&pre)[NPRE]) {
  using TR = EpiTraits<EPI, BM, BN>;
  static_assert(!WT || EPI == EPI_BIAS || EPI == EPI_BF16, "write-through stores: plain bf16 epilogues only");
  constexpr int LDC = BN * TR::ES + 16;
  constexpr int CPR8 = BN / 8, NCH = BM * CPR8 / NT;
  constexpr bool PRE = TR::ELEM && TR::F32S && (BM * CPR8) % NT == 0 && NCH <= 8;
  if constexpr (!TR::F32S) {
    constexpr int CPR = BN / 8;  // 16-byte chunks (8 bf16) per row
    bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
#pragma unroll 4
    for (int id = tid; id < BM * CPR; id += NT) {
      const int r = id / CPR, cc = id - r * CPR;
      const int m = m0 + r;
      if (m >= p.M) break;  // rows ascend with id
      const uint4 u = *reinterpret_cast<const uint4*>(smem + r * LDC + cc * 16);
      const int n = n0 + cc * 8;
      if constexpr (EPI == EPI_BIAS_GELU) {
        // GELU on the bf16-rounded pre-activation, exactly what the backward re-reads (no aux: a
        // forward without autograd -- the teacher, evaluation -- keeps only the activation)
        if (p.aux) *reinterpret_cast<uint4*>(p.aux + (size_t)m * p.ldaux + n) = u;
        uint4 y;
        y.x = pack_bf2(gelu_erf(lo_bf(u.x)), gelu_erf(hi_bf(u.x)));
        y.y = pack_bf2(gelu_erf(lo_bf(u.y)), gelu_erf(hi_bf(u.y)));
        y.z = pack_bf2(gelu_erf(lo_bf(u.z)), gelu_erf(hi_bf(u.z)));
        y.w = pack_bf2(gelu_erf(lo_bf(u.w)), gelu_erf(hi_bf(u.w)));
        *reinterpret_cast<uint4*>(C + (size_t)m * p.ldc + n) = y;
      } else if constexpr (WT) {
        // (the resource from kernel arguments only: uniform; < 2 GiB checked by the launcher)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, u),
                                               __builtin_amdgcn_make_buffer_rsrc(p.C, 0, 0x7fffffff, 0x00020000),
                                               (int)(((size_t)m * p.ldc + n) * 2), 0, LN2_SC1);
      } else {
        *reinterpret_cast<uint4*>(C + (size_t)m * p.ldc + n) = u;
      }
    }
    if constexpr (WT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing thread drains
  } else if constexpr (EPI == EPI_F32) {
    f32_epilogue<BM, BN, NT>(p, smem, LDC, m0, n0, tid);
  } else {
    // 8 fp32 per chunk: two float4 LDS reads, then one 16-byte load / store per global stream
    constexpr int CPR = BN / 8;
    constexpr bool CS_OK = NT % CPR == 0;  // a thread keeps one column chunk for the whole tile
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // column sums of this thread's rows (p.colsum)
    // one chunk: 8 fp32 of row r from LDS, finished with the 16-byte aux / residual chunk u
    auto chunk = [&](int r, int cc, const uint4& u) {
      const int m = m0 + r;
      const float4 va = *reinterpret_cast<const float4*>(smem + r * LDC + cc * 32);
      const float4 vb = *reinterpret_cast<const float4*>(smem + r * LDC + cc * 32 + 16);
      float v[8] = {va.x, va.y, va.z, va.w, vb.x, vb.y, vb.z, vb.w};
      const int n = n0 + cc * 8;
      if constexpr (EPI == EPI_GELU_BWD) {
        const uint32_t uw[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] *= gelu_erf_grad(lo_bf(uw[e]));
          v[2 * e + 1] *= gelu_erf_grad(hi_bf(uw[e]));
        }
        if (p.aux_out) {
          gelu_remat(p, m, n, make_uint2(u.x, u.y));
          gelu_remat(p, m, n + 4, make_uint2(u.z, u.w));
        }
      } else {  // EPI_ADD
        const uint32_t rw[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] += lo_bf(rw[e]);
          v[2 * e + 1] += hi_bf(rw[e]);
        }
      }
      bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
      const uint4 o = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7]));
      *reinterpret_cast<uint4*>(C + (size_t)m * p.ldc + n) = o;
      // the sums are of the stored (bf16) values: what a separate column sum would read
      if constexpr (CS_OK) {
        const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) { cs[2 * e] += lo_bf(ow[e]); cs[2 * e + 1] += hi_bf(ow[e]); }
      }
    };
    if constexpr (PRE) {
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int id = tid + k * NT, r = id / CPR, cc = id - r * CPR;
        if (m0 + r < p.M) chunk(r, cc, pre[k]);
      }
    } else {
#pragma unroll 2
      for (int id = tid; id < BM * CPR; id += NT) {
        const int r = id / CPR, cc = id - r * CPR;
        const int m = m0 + r;
        if (m >= p.M) break;
        const uint4 u = EPI == EPI_GELU_BWD ? *reinterpret_cast<const uint4*>(p.aux + (size_t)m * p.ldaux + n0 + cc * 8)
                                            : *reinterpret_cast<const uint4*>(p.res + (size_t)m * p.ldres + n0 + cc * 8);
        chunk(r, cc, u);
      }
    }
    if (CS_OK && p.colsum) {
      // per-tile column partials [tiles_m][N] (fixed order: deterministic), finalised by the
      // batched column-sum launch at the end of the backward (norm.hip fd_colsum_batched)
      constexpr int G = CS_OK ? NT / CPR : 1;  // threads sharing a column chunk
      float* red = reinterpret_cast<float*>(smem);
      __syncthreads();  // every thread is done reading the staged tile
      const int cc = tid % CPR, g = tid / CPR;
#pragma unroll
      for (int e = 0; e < 8; ++e) red[g * BN + cc * 8 + e] = cs[e];
      __syncthreads();
      for (int c = tid; c < BN; c += NT) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < G; ++i) s += red[i * BN + c];
        p.colsum[(size_t)(m0 / BM) * p.N + n0 + c] = s;
      }
    }
  }
}

// ---------------------------------------------------------------- LayerNorm epilogues
// EPI_LN / EPI_LN_BWD (FdLnEpi, adam_epi.h).  The tile is parked in LDS as fp32, then CPR
// consecutive lanes own one tile row (8 columns each) for the element math; the row's two
// partial statistics over this tile's BN columns reduce in a CPR-lane butterfly (every lane
// ends with the same bits) and are published to stats[tm][tn][2][row].  Every tile of the row
// block then reads all tiles_n partials and merges them in the same fixed order -- so each
// normalises its slice with bitwise the same row mean / rstd.
//
// Exchange (no device-scope fence -- a full L2 writeback per block on the 8 non-coherent XCD
// L2s; no arrival counter): each statistic is an 8-byte granule {tag, value} written by ONE
// agent-scope relaxed atomic store (global store with the coherence bit, not kept in the XCD's
// L2), and the readers poll the granules themselves with agent-scope atomic loads until every
// tag is this launch's -- the data is the flag, so there is nothing to order.  The tag is
// epoch * FD_LN_XSITES + xsite + 1: the epoch is advanced once per model forward by an earlier
// launch (norm.hip emb_fwd_kernel) and every LN launch of that forward / backward passes its own
// call site, so stale granules of earlier launches never match and no launch needs a "last
// block" fan-in to advance anything (the old per-launch done counter cost ~2 us per call).
// Progress: a row block's tiles are consecutive logical tiles, walked in order per XCD
// (xcd_remap), and the grid is one resident round.  The poll is bounded by the wall clock
// (0.25 s, never reached in a healthy launch): a timeout sets ln.err, which the host treats as
// fatal (ops/kernels.py check_ln_error) -- the tile's statistics are then wrong.
DEV void st_gran(uint64_t* p, uint32_t tag, float v) {
  __hip_atomic_store(p, ((uint64_t)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV uint64_t ld_gran(uint64_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DEV float gran_val(uint64_t g) { return __uint_as_float((uint32_t)g); }

template <int CPR>
DEV float row_sum(float v) {  // butterfly over the CPR lanes of a row: identical bits in each
#pragma unroll
  for (int o = 1; o < CPR; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

DEV void load8f(const float* p, float (&f)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
DEV void unpack8bf(const uint4& u, float (&f)[8]) {
  f[0] = lo_bf(u.x); f[1] = hi_bf(u.x); f[2] = lo_bf(u.y); f[3] = hi_bf(u.y);
  f[4] = lo_bf(u.z); f[5] = hi_bf(u.z); f[6] = lo_bf(u.w); f[7] = hi_bf(u.w);
}
DEV uint4 pack8bf(const float (&f)[8]) {
  return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
}

constexpr int LN_MAXK = 4;  // column tiles per row block <= LN_MAXK * (BN / 8)
// Largest LayerNorm-fused grid: one round of the 256 CUs, every tile resident at once (no row
// block waits on a tile that cannot be dispatched yet).  Measured: at two rounds' worth of tiles
// (bs64 x seq256 packed, 492 tiles) the fused GEMMs lose to GEMM + LN kernels even with two
// 72 KiB blocks per CU (5.99 vs 5.78 ms/step, profiles/r2_ab_fused_ln_kd_seq256.txt), so
// larger grids take the separate LayerNorm kernels (ops/kernels.py ln_fusable mirrors this).
constexpr int LN_MAX_TILES = 256;

// The per-thread operands of the LayerNorm epilogue's element math (a thread owns IT rows x 8
// columns): residual, backward z / mean / rstd, dropout-hash rows, gamma, the exchange tag --
// LDS-DMA'd under the last K tiles (ln_dma), or loaded right after the K loop (their ring's
// inline-asm waits would count VGPR loads issued inside the loop as ring tiles).
template <int IT>
struct LnPre {
  uint4 res_v[IT], z_v[IT];
  float mrow[IT], rrow[IT];
  int hrow_v[IT];
  float g[8], bt[8];  // gamma / beta (forward) of this thread's 8 columns
  uint32_t tag;
};

template <int BM, int BN, bool BWD, int NT>
DEV LnPre<BM * (BN / 8) / NT> ln_prefetch(const GemmParams& p, int tm, int tn, int tid) {
  constexpr int CPR = BN / 8, IT = BM * CPR / NT;
  const FdLnEpi& L = p.ln;
  const int m0 = tm * BM, N = p.N;
  const int n = tn * BN + 8 * (tid % CPR);
  LnPre<IT> pre;
  pre.tag = (uint32_t)__hip_atomic_load(L.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * FD_LN_XSITES + L.xsite + 1u;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int mc = min(m0 + (tid + it * NT) / CPR, p.M - 1);
    pre.res_v[it] = *reinterpret_cast<const uint4*>(p.res + (size_t)mc * p.ldres + n);
    if constexpr (BWD) {
      pre.z_v[it] = *reinterpret_cast<const uint4*>(L.z + (size_t)mc * N + n);
      pre.mrow[it] = L.mean[mc];
      pre.rrow[it] = L.rstd[mc];
    }
    pre.hrow_v[it] = (L.thr && L.row_map) ? L.row_map[mc] : mc;
  }
  load8f(L.gamma + n, pre.g);
  if constexpr (!BWD) load8f(L.beta + n, pre.bt);
  return pre;
}

// The same operands LDS-DMA'd by the LDS-DMA kernels into the two ring slots their last K-tile
// pair leaves free (gemm_tile_at, EPI_LN / EPI_LN_BWD, S >= 6): the loads land under that pair's
// MFMAs instead of stalling the epilogue (round 3 stamps: 2-4 us of epilogue before the
// rendezvous, mostly this latency).  Region layout (dst): [0, 16 K) the residual tile, [16 K, 32 K)
// z (backward), then 1 KiB pieces: gamma | beta, mean | rstd (backward), the dropout-hash rows.
// Rows past M re-read row M - 1 (never stored); per-row scalars need M % 4 == 0 (caller).  Each
// wave issues ln_dma_ops() DMAs (vmcnt is per wave).
constexpr int LN_DMA_MISC = 32768;
DEV bool ln_dma_rowmap(const FdLnEpi& L) { return L.thr != 0 && L.row_map != nullptr; }

template <bool BWD>
DEV int ln_dma_ops(const FdLnEpi& L, int wid, int ppw) {
  return ppw * (BWD ? 2 : 1) + (wid == 0) + (BWD && wid == 1) + (wid == 2 && ln_dma_rowmap(L));
}

template <int BM, int BN, bool BWD, int NW>
DEV void ln_dma(const GemmParams& p, int tm, int tn, char* dst, int wid, int lane) {
  constexpr int PIECES = BM * BN * 2 / 1024, PPW = PIECES / NW;
  static_assert(BN * 2 == 128 && PIECES % NW == 0, "ln prefetch tile");
  const FdLnEpi& L = p.ln;
  const int m0 = tm * BM, n0 = tn * BN;
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int piece = wid * PPW + i;
    const int mc = min(m0 + piece * 8 + (lane >> 3), p.M - 1), c = lane & 7;
    glds16(p.res + (size_t)mc * p.ldres + n0 + c * 8, dst + piece * 1024);
    if constexpr (BWD) glds16(L.z + (size_t)mc * p.N + n0 + c * 8, dst + 16384 + piece * 1024);
  }
  char* misc = dst + LN_DMA_MISC;
  if (wid == 0) {  // lanes 0-15 gamma, 16-31 beta (forward)
    if (lane < 16) glds16(L.gamma + n0 + 4 * lane, misc);
    else if (!BWD && lane < 32) glds16(L.beta + n0 + 4 * (lane - 16), misc);
  }
  if (BWD && wid == 1) {  // lanes 0-31 mean, 32-63 rstd: 4 rows per lane
    const int r = m0 + 4 * (lane & 31);
    if (r < p.M) glds16((lane < 32 ? L.mean : L.rstd) + r, misc + 1024);
  }
  if (wid == 2 && ln_dma_rowmap(L)) {
    const int r = m0 + 4 * lane;
    if (lane < BM / 4 && r < p.M) glds16(L.row_map + r, misc + 2048);
  }
}

template <int BM, int BN, bool BWD, int NT>
DEV LnPre<BM * (BN / 8) / NT> ln_from_lds(const GemmParams& p, int tm, int tn, int tid, const char* src) {
  constexpr int CPR = BN / 8, IT = BM * CPR / NT;
  const FdLnEpi& L = p.ln;
  const int m0 = tm * BM, cc = tid % CPR;
  const char* misc = src + LN_DMA_MISC;
  LnPre<IT> pre;
  pre.tag = (uint32_t)__hip_atomic_load(L.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * FD_LN_XSITES + L.xsite + 1u;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int r = (tid + it * NT) / CPR;
    pre.res_v[it] = *reinterpret_cast<const uint4*>(src + r * 128 + cc * 16);
    if constexpr (BWD) {
      pre.z_v[it] = *reinterpret_cast<const uint4*>(src + 16384 + r * 128 + cc * 16);
      pre.mrow[it] = reinterpret_cast<const float*>(misc + 1024)[r];
      pre.rrow[it] = reinterpret_cast<const float*>(misc + 1536)[r];
    }
    pre.hrow_v[it] = ln_dma_rowmap(L) ? reinterpret_cast<const int*>(misc + 2048)[r] : min(m0 + r, p.M - 1);
  }
  load8f(reinterpret_cast<const float*>(misc) + 8 * cc, pre.g);
  if constexpr (!BWD) load8f(reinterpret_cast<const float*>(misc + 256) + 8 * cc, pre.bt);
  return pre;
}

// The LayerNorm epilogue in two steps: ln_park (each wave's accumulators, + bias in the forward,
// into the fp32 LDS tile [BM][BN]) and ln_finish (the element math, the row-statistics exchange,
// the normalisation and the stores).  ln_epilogue = both; the two-K-half kernel parks only the
// waves that hold its final columns (gemm_ln2_kernel).
template <int BM, int BN, int TM, int TN, bool BWD>
DEV void ln_park(const GemmParams& p, const f32x4 (&acc)[TM / 16][TN / 16], char* smem, int n0, int wr, int wc,
                 int lane) {
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int LDC = BN * 4 + 16;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int r = wr * TM + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int c = wc * TN + j * 16 + 4 * (lane >> 4);
      float4 v = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      if constexpr (!BWD) {
        const float4 b = *reinterpret_cast<const float4*>(p.bias + n0 + c);
        v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
      }
      *reinterpret_cast<float4*>(smem + r * LDC + c * 4) = v;
    }
  }
}


template <int BM, int BN, bool BWD, int NT>
DEV void ln_finish(const GemmParams& p, char* smem, int tm, int tn, int lane, int tid,
                   const LnPre<BM * (BN / 8) / NT>& pre) {
  constexpr int LDC = BN * 4 + 16;
  constexpr int CPR = BN / 8;            // lanes per row (8 columns each)
  constexpr int IT = BM * CPR / NT;      // rows per thread
  static_assert(CPR >= 2 && CPR <= 64 && (CPR & (CPR - 1)) == 0 && NT % CPR == 0 && IT * NT == BM * CPR, "ln tile");
  const FdLnEpi& L = p.ln;
  const int m0 = tm * BM, n0 = tn * BN, tiles_n = p.N / BN, N = p.N;
  const int cc = tid % CPR, n = n0 + 8 * cc;
  const uint32_t tag = pre.tag;
  uint4 z_v[IT];
  const uint4* res_v = pre.res_v;
  const float* mrow = pre.mrow;
  const float* rrow = pre.rrow;
  const int* hrow_v = pre.hrow_v;
#pragma unroll
  for (int it = 0; it < IT; ++it) z_v[it] = pre.z_v[it];
  const float* g = pre.g;
  __syncthreads();
  const bool drop = L.thr != 0;
  const uint32_t seed = drop ? hash32(L.seed_ptr[0], L.site) : 0u;
  uint64_t* stats = L.stats + (size_t)(tm * tiles_n) * 2 * BM;  // [tn][2][BM] of this row block
  float zv[IT][8], xv[IT][8];  // forward: z;  backward: gamma dy (zv) and xhat (xv)
  float cg[8] = {}, cb[8] = {};  // backward column partials: dgamma, dbeta
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int r = (tid + it * NT) / CPR, m = m0 + r;
    float v[8];
    load8f(reinterpret_cast<const float*>(smem + r * LDC) + 8 * cc, v);
    float rr[8];
    unpack8bf(res_v[it], rr);
    if constexpr (!BWD) {
      if (drop) {
        const size_t hrow = (size_t)(unsigned)hrow_v[it];
        const uint32_t kb = drop_keep_bits<8>(seed, (uint32_t)(hrow * N + n), L.thr);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (kb >> e) & 1u ? v[e] * L.dscale : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += rr[e];
      // the normalisation runs on the bf16-rounded sum: exactly what the backward re-reads
      // (stored after the rendezvous: the statistics publish drains only their own stores)
      z_v[it] = pack8bf(v);
      unpack8bf(z_v[it], zv[it]);
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) s += zv[it][e];
      const float mt = row_sum<CPR>(s) * (1.f / BN);
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = zv[it][e] - mt; q += d * d; }
      q = row_sum<CPR>(q);
      if (cc == 0) { st_gran(stats + (size_t)tn * 2 * BM + r, tag, mt); st_gran(stats + (size_t)(tn * 2 + 1) * BM + r, tag, q); }
      if (L.z && m < p.M) *reinterpret_cast<uint4*>(L.z + (size_t)m * N + n) = z_v[it];  // (before the wait)
    } else {
      float zz[8];
      unpack8bf(z_v[it], zz);
      const float mean = mrow[it], rstd = rrow[it];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dy = v[e] + rr[e];
        const float xh = (zz[e] - mean) * rstd;
        xv[it][e] = xh;
        zv[it][e] = g[e] * dy;
        s1 += zv[it][e];
        s2 += zv[it][e] * xh;
        if (m < p.M) { cg[e] += dy * xh; cb[e] += dy; }
      }
      s1 = row_sum<CPR>(s1);
      s2 = row_sum<CPR>(s2);
      if (cc == 0) { st_gran(stats + (size_t)tn * 2 * BM + r, tag, s1); st_gran(stats + (size_t)(tn * 2 + 1) * BM + r, tag, s2); }
    }
  }
  // backward column partials (lanes of a wave with the same column chunk, then the waves):
  // dgamma / dbeta need no row statistics, so they are reduced and stored while the other
  // tiles' granules are in flight; dbias follows the normalisation
  constexpr int NWV = NT / 64;
  float* red = reinterpret_cast<float*>(smem);  // [2][NWV][BN]
  auto park = [&](float (&a)[8], int slot) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1) a[e] += __shfl_xor(a[e], o, 64);
    }
    if (lane < CPR) {
      float* dst = red + (slot * NWV + (tid >> 6)) * BN + 8 * lane;
      *reinterpret_cast<float4*>(dst) = make_float4(a[0], a[1], a[2], a[3]);
      *reinterpret_cast<float4*>(dst + 4) = make_float4(a[4], a[5], a[6], a[7]);
    }
  };
  auto flush = [&](int nslot, int w30) {  // colpart rows w30 .. w30 + nslot - 1 from slots 0 ..
    for (int i = tid; i < nslot * BN; i += NT) {
      const int sl = i / BN, c = i % BN;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) v += red[(sl * NWV + w) * BN + c];
      L.colpart[((size_t)tm * 3 + w30 + sl) * N + n0 + c] = v;
    }
  };
  if constexpr (BWD) {
    __syncthreads();  // the staged tile has been read
    park(cg, 0);
    park(cb, 1);
    __syncthreads();
    flush(2, 0);
  }
  // this lane's share of the tiles_n partials of its rows (tiles cc, cc + CPR, ...): poll the
  // granules until every tag is this launch's (wave-uniform exit)
  float2 st[IT][LN_MAXK];
  FD_STAMP(3);
  const PfRegs pfr = pf_issue<NT>(L, tid);
  {
    // diag 64 (tests only): wait for a tag no launch writes -> the timeout path
    const uint32_t want = (p.diag & 64) ? tag + 1u : tag;
    const uint64_t t0 = wall_clock64();  // 100 MHz
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int r = (tid + it * NT) / CPR;
#pragma unroll
        for (int i = 0; i < LN_MAXK; ++i) {
          const int t = cc + i * CPR;
          if (t < tiles_n) {
            const uint64_t a = ld_gran(stats + (size_t)t * 2 * BM + r);
            const uint64_t b = ld_gran(stats + (size_t)(t * 2 + 1) * BM + r);
            ok &= (uint32_t)(a >> 32) == want && (uint32_t)(b >> 32) == want;
            st[it][i] = make_float2(gran_val(a), gran_val(b));
          } else {
            st[it][i] = make_float2(0.f, 0.f);
          }
        }
      }
      if (__all(ok) || (p.diag & 16)) break;  // (diag 16: timing only -- no wait, wrong statistics)
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > 25000000ull) {  // 0.25 s: never in a healthy launch
        if (lane == 0) __hip_atomic_fetch_or(L.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  FD_STAMP(4);
  const float* bt = pre.bt;
  float cd[8] = {};  // backward: dbias partials
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int r = (tid + it * NT) / CPR, m = m0 + r;
    // the row butterfly over the lanes' partials: a fixed order, the same in every tile
    const float2 (&st_r)[LN_MAXK] = st[it];
    const size_t off = (size_t)min(m, p.M - 1) * N + n;
    if constexpr (!BWD) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < LN_MAXK; ++i) s += st_r[i].x;
      const float mean = row_sum<CPR>(s) / tiles_n;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < LN_MAXK; ++i) {
        const float d = st_r[i].x - mean;
        if (cc + i * CPR < tiles_n) q += st_r[i].y + BN * d * d;
      }
      const float rstd = rsqrtf(row_sum<CPR>(q) / N + L.eps);
      float y[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) y[e] = (zv[it][e] - mean) * rstd * g[e] + bt[e];
      if (m < p.M) {
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(p.C) + off) = pack8bf(y);
        if (tn == 0 && cc == 0) { L.mean[m] = mean; L.rstd[m] = rstd; }
      }
    } else {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int i = 0; i < LN_MAXK; ++i) { a += st_r[i].x; b += st_r[i].y; }
      const float s1 = row_sum<CPR>(a) / N, s2 = row_sum<CPR>(b) / N;
      float dz[8], dx[8];
      const size_t hrow = (size_t)(unsigned)hrow_v[it];
      const uint32_t kb = drop ? drop_keep_bits<8>(seed, (uint32_t)(hrow * N + n), L.thr) : 0xffu;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dz[e] = rrow[it] * (zv[it][e] - s1 - xv[it][e] * s2);
        dx[e] = drop ? ((kb >> e) & 1u ? dz[e] * L.dscale : 0.f) : dz[e];
      }
      if (m < p.M) {
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(p.C) + off) = pack8bf(dz);
        if (drop && L.dx) *reinterpret_cast<uint4*>(L.dx + off) = pack8bf(dx);
#pragma unroll
        for (int e = 0; e < 8; ++e) cd[e] += dx[e];
      }
    }
  }
  if constexpr (BWD) {
    __syncthreads();  // slots 0 / 1 have been flushed
    park(cd, 0);
    __syncthreads();
    flush(1, 2);
  }
  pf_consume(pfr);
}

template <int BM, int BN, int TM, int TN, bool BWD, int NT>
DEV void ln_epilogue(const GemmParams& p, const f32x4 (&acc)[TM / 16][TN / 16], char* smem, int tm, int tn,
                     int wr, int wc, int lane, int tid, const LnPre<BM * (BN / 8) / NT>& pre) {
  ln_park<BM, BN, TM, TN, BWD>(p, acc, smem, tn * BN, wr, wc, lane);
  ln_finish<BM, BN, BWD, NT>(p, smem, tm, tn, lane, tid, pre);
}

// ---------------------------------------------------------------- two-K-half LayerNorm tiles
// gemm_ln2_kernel: the blocks s = 0, 1 of a pair each run HALF of the K loop of one 128 x 128
// product tile (twice the MFMA work per staged byte of a 128 x 64 tile, half the K steps), then
// trade the fp32 partial of the 64-column half they do not finish: block s finishes columns
// [64 s, 64 s + 64) -- LayerNorm tile tn = 2 tnp + s of the plain 128 x 64 layout, so the
// row-statistics exchange and everything after it is ln_finish's.  Wave (wr, wc) holds rows
// 32 wr.. and columns 64 wc.. of the product (TM = 32, TN = 64); the waves with wc != s send,
// the partner's waves with the same (wr, wc) receive -- the same fragment layout, so the sum is
// element by element, no shuffles.  Final = own + partner's partial in both blocks: the same
// IEEE sum either way (addition commutes), independent of timing.
// Hand-off (cdna_hip_programming.md Guideline 16, write-through form; one block per CU): the
// payload goes out with 16-byte sc1 (write-through) stores, every storing wave drains them
// (vmcnt(0)), a workgroup barrier, then ONE lane stores the {tag, 1} flag granule with an
// agent-scope atomic store; each receiving wave polls the partner's flag with agent-scope atomic
// loads and reads the payload with sc1 loads only after its own poll has matched.  The tag is the
// LayerNorm exchange's (epoch * FD_LN_XSITES + xsite + 1): stale flags never match.

DEV __amdgpu_buffer_rsrc_t ln2_rsrc(const FdLnEpi& L) {
  // the whole exchange buffer, from kernel arguments only (wave-uniform: no waterfall loops);
  // every per-block / per-wave part of an address goes in the 32-bit voffset
  return __builtin_amdgcn_make_buffer_rsrc(L.xbuf, 0, 0x7fffffff, 0x00020000);
}
template <int MI, int NI>
constexpr int ln2_wave_bytes() { return MI * NI * 64 * 16; }

template <int MI, int NI>
DEV void ln2_send(const GemmParams& p, const f32x4 (&acc)[MI][NI], int pair, int s, int wr, int wc, int lane,
                  uint32_t tag) {
  const FdLnEpi& L = p.ln;
  if (wc != s) {  // these columns are the partner's
    const __amdgpu_buffer_rsrc_t rs = ln2_rsrc(L);
    const int base = ((pair * 2 + s) * 4 + wr) * ln2_wave_bytes<MI, NI>() + lane * 16;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, acc[i][j]), rs,
                                               base + (i * NI + j) * 64 * 16, 0, LN2_SC1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its own stores
  }
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(L.xflag + pair * 2 + s, ((uint64_t)tag << 32) | 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MI, int NI>
DEV void ln2_recv(const GemmParams& p, f32x4 (&acc)[MI][NI], int pair, int s, int wc, int wr, int lane,
                  uint32_t tag) {
  const FdLnEpi& L = p.ln;
  if (wc != s) return;
  uint64_t* fl = L.xflag + pair * 2 + (1 - s);
  const uint32_t want = (p.diag & 64) ? tag + 1u : tag;
  const uint64_t t0 = wall_clock64();
  for (;;) {
    const uint64_t f = __hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)(f >> 32) == want) break;
    __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > 25000000ull) {  // 0.25 s: never in a healthy launch
      if (lane == 0) __hip_atomic_fetch_or(L.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the poll)
  const __amdgpu_buffer_rsrc_t rs = ln2_rsrc(L);
  const int base = ((pair * 2 + (1 - s)) * 4 + wr) * ln2_wave_bytes<MI, NI>() + lane * 16;
  f32x4 other[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
      other[i][j] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, base + (i * NI + j) * 64 * 16, 0, LN2_SC1));
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = acc[i][j] + other[i][j];
}

// Scheduling hints for one K tile: the first 32-deep fragment set's ds_reads,
// then each of its MFMAs followed by RPM of the second set's ds_reads (their
// latency hides under the MFMA pipe), then the second set's MFMAs.
template <int N, int RPM>
DEV void sched_interleave() {
  if constexpr (N > 0) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, RPM, 0);  // DS read
    sched_interleave<N - 1, RPM>();
  }
}
template <int R, int M>
DEV void sched_ktile() {
  __builtin_amdgcn_sched_group_barrier(0x100, R, 0);
  sched_interleave<M, (R + M - 1) / M>();
  __builtin_amdgcn_sched_group_barrier(0x008, M, 0);
}

template <int N>
DEV void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Runtime count of ops allowed in flight (vmcnt needs an immediate): 0 .. 7.
DEV void wait_ops(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<1>(); break;
    case 2: wait_vm<2>(); break;
    case 3: wait_vm<3>(); break;
    case 4: wait_vm<4>(); break;
    case 5: wait_vm<5>(); break;
    case 6: wait_vm<6>(); break;
    default: wait_vm<7>(); break;
  }
}

// Counted wait for "all but the youngest n*L LDS-DMA ops" (n = tiles still allowed in flight).
template <int L, int MAXN>
DEV void wait_tiles(int n) {
  if constexpr (MAXN >= 4) { if (n >= 4) { wait_vm<4 * L>(); return; } }
  if constexpr (MAXN >= 3) { if (n >= 3) { wait_vm<3 * L>(); return; } }
  if constexpr (MAXN >= 2) { if (n >= 2) { wait_vm<2 * L>(); return; } }
  if constexpr (MAXN >= 1) { if (n >= 1) { wait_vm<L>(); return; } }
  wait_vm<0>();
}

template <int BM, int BN, bool AK, bool BKM, int EPI, int WM, int WN, int S, int BK = BKT>
struct GemmCfg {
  static constexpr int NW = WM * WN;
  using OA = Operand<BM, AK, NW, BK>;
  using OB = Operand<BN, BKM, NW, BK>;
  static constexpr int BUF = OA::BYTES + OB::BYTES;
  // DIRECT fp32 tiles are staged one wave-row band (BM / WM rows) at a time
  static constexpr int EPI_BYTES = EpiTraits<EPI, BM, BN>::DIRECT ? (BM / WM) * (BN * 4 + 16)
                                                                   : EpiTraits<EPI, BM, BN>::BYTES;
  static constexpr int SMEM = S * BUF > EPI_BYTES ? S * BUF : EPI_BYTES;
  // (the accumulator-direct fp32 epilogue serves only the all-layer weight-gradient launch)
  static constexpr bool VALID = SMEM <= LDS_MAX && !EpiTraits<EPI, BM, BN>::DIRECT &&
                                (!EpiTraits<EPI, BM, BN>::LN || EpiTraits<EPI, BM, BN>::F32S) &&
                                (BKM || BN % 64 == 0) &&
                                (AK || BM % 64 == 0) &&
                                (BM / WM) % 16 == 0 && (BN / WN) % 16 == 0 &&
                                OA::PER_WAVE * NW * 1024 == OA::BYTES && OB::PER_WAVE * NW * 1024 == OB::BYTES;
};

// Grouped launch (weight gradients): a second problem with the same K and kinds whose
// tiles follow the first's in the logical tile order, so two dW GEMMs that become ready
// together (lin1 + lin2, out_lin + qkv) fill the chip as one grid instead of two
// split-K launches each with its own slab round trip.
struct GemmGroup {
  GemmParams q;   // second problem (used when ntiles0 < total tiles)
  int ntiles0;    // tiles of the first problem
  int ntiles;     // tiles of both
};

#ifndef FD_GEMM_SCHED
#define FD_GEMM_SCHED 1
#endif

// One output tile (tm, tn) of problem p: the K loop over the LDS-DMA ring, then the epilogue.
template <int BM, int BN, bool AK, bool BKM, int EPI, int WM, int WN, int S, int BK = BKT, bool WT = false>
DEV void gemm_tile_at(const GemmParams& p, int tm, int tn, char* smem) {
  const int tm_ = tm, tn_ = tn;
  using G = GemmCfg<BM, BN, AK, BKM, EPI, WM, WN, S, BK>;
  constexpr int KS = BK / 32;  // 32-deep MFMA k-steps per ring slot
  using OA = typename G::OA;
  using OB = typename G::OB;
  constexpr int NW = G::NW;
  constexpr int TM = BM / WM, TN = BN / WN;  // per-wave tile
  constexpr int MI = TM / 16, NI = TN / 16;  // 16x16 sub-tiles per wave
  constexpr int BUF = G::BUF;
  constexpr int L = OA::PER_WAVE + OB::PER_WAVE;  // DMA ops per wave per K tile
  static_assert(S >= 2 && S <= 6, "ring depth");
  static_assert((S - 2) * L <= 63, "vmcnt is 6 bits");
  constexpr bool SCHED = FD_GEMM_SCHED;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.z * p.k_split;
  const int nk = p.k_split / BK;

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int t) {
    char* b = smem + (t % S) * BUF;
    OA::stage(p.A, p.lda, m0, kbeg + t * BK, p.M, b, wid, lane);
    OB::stage(p.B, p.ldb, n0, kbeg + t * BK, p.N, b + OA::BYTES, wid, lane);
  };
  bf16x8 a0[MI], b0[NI], a1[MI], b1[NI];
  // column sums of A (EPI_F32 acol): lane l's A fragments hold 8 k values of column m = l % 16
  // of each 16-column block; only the first column block's tiles and their wc == 0 waves sum
  const bool acs = EPI == EPI_F32 && p.acol != nullptr && tn == 0 && wc == 0;
  float asum[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) asum[i] = 0.f;
  auto sum_a = [&]() {
    if constexpr (EPI == EPI_F32) {
      if (acs) {
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          float s = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            s += bf2f((uint16_t)a0[i][e]);
            if constexpr (KS == 2) s += bf2f((uint16_t)a1[i][e]);
          }
          asum[i] += s;
        }
      }
    }
  };
  auto read_frags = [&](const char* cur) {
#pragma unroll
    for (int i = 0; i < MI; ++i) a0[i] = OA::frag(cur, wr * TM + i * 16, 0, lane);
#pragma unroll
    for (int j = 0; j < NI; ++j) b0[j] = OB::frag(cur + OA::BYTES, wc * TN + j * 16, 0, lane);
    if constexpr (KS == 2) {
#pragma unroll
      for (int i = 0; i < MI; ++i) a1[i] = OA::frag(cur, wr * TM + i * 16, 1, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) b1[j] = OB::frag(cur + OA::BYTES, wc * TN + j * 16, 1, lane);
    }
  };
  auto mfmas = [&]() {
    if constexpr (!SCHED) __builtin_amdgcn_s_setprio(1);  // (s_setprio would split the scheduling region)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(b0[j], a0[i], acc[i][j]);
    if constexpr (KS == 2) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(b1[j], a1[i], acc[i][j]);
    }
    if constexpr (!SCHED) __builtin_amdgcn_s_setprio(0);
  };

  // LayerNorm epilogue operands LDS-DMA'd under the last two K-tile pairs (ln_dma): S >= 6 rings
  // whose K tiles are a whole number of rings, so the pair before last frees slots 0 and 1
  constexpr bool LNPF = EpiTraits<EPI, BM, BN>::LN && S >= 6 && BN == 64 && (BM * BN * 2 / 1024) % NW == 0 &&
                        2 * BUF >= LN_DMA_MISC + 3072;
  const bool lnpf = LNPF && nk % S == 0 && nk >= S && p.M % 4 == 0 && !(p.diag & (1 | 128));
  int e_ops = 0;  // this wave's epilogue DMAs in flight (younger than every ring tile)
  if constexpr (S < 6) {
#pragma unroll
    for (int t = 0; t < S - 1; ++t)
      if (t < nk) issue(t);

    for (int kt = 0; kt < nk; ++kt) {
      // this wave's DMA for tile kt has landed (younger tiles stay in flight) ...
      wait_tiles<L, S - 2>(min(S - 2, nk - 1 - kt));
      // ... and everyone's has; everyone is also done reading tile kt-1's slot.
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (FD_GEMM_STAMPS && kt == 0) FD_STAMP(1);
      if (kt + S - 1 < nk && !(p.diag & 1)) issue(kt + S - 1);
      read_frags(smem + (kt % S) * BUF);
      mfmas();
      sum_a();
      if constexpr (SCHED) sched_ktile<(MI * (AK ? 1 : 2) + NI * (BKM ? 1 : 2)) * KS / 2, MI * NI * KS / 2>();
    }
  } else {
    // Two K tiles per barrier (S >= 6): the slots of the pair read in the previous step are
    // refilled after ONE barrier, S - 4 tiles stay in flight across it -- half the barriers
    // and waits of the loop above for the same bytes in flight.
#pragma unroll
    for (int t = 0; t < S - 2; ++t)
      if (t < nk) issue(t);

    for (int kt = 0; kt < nk; kt += 2) {
      const int issued = min(nk, S - 2 + kt);
      const int need = min(kt + 2, nk);
      if (LNPF && lnpf && kt == nk - 2) {
        wait_ops(e_ops);  // the last pair's tiles; only the epilogue DMAs stay in flight
      } else {
        wait_tiles<L, S - 4>(min(S - 4, max(0, issued - need)));
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (FD_GEMM_STAMPS && kt == 0) FD_STAMP(1);
      if (!(p.diag & 1)) {
        if (kt + S - 2 < nk) issue(kt + S - 2);  // slot of tile kt-2
        if (kt + S - 1 < nk) issue(kt + S - 1);  // slot of tile kt-1
      }
      if constexpr (LNPF) {
        if (lnpf && kt == nk - 4) {  // slots 0 / 1 (tiles nk - 6, nk - 5) were read last pair; no refill
          ln_dma<BM, BN, EPI == EPI_LN_BWD, NW>(p, tm_, tn_, smem, wid, lane);
          e_ops = ln_dma_ops<EPI == EPI_LN_BWD>(p.ln, wid, (BM * BN * 2 / 1024) / NW);
        }
      }
      read_frags(smem + (kt % S) * BUF);
      mfmas();
      sum_a();
      if constexpr (SCHED) sched_ktile<(MI * (AK ? 1 : 2) + NI * (BKM ? 1 : 2)) * KS / 2, MI * NI * KS / 2>();
      if (kt + 1 < nk) {
        read_frags(smem + ((kt + 1) % S) * BUF);
        mfmas();
        sum_a();
        if constexpr (SCHED) sched_ktile<(MI * (AK ? 1 : 2) + NI * (BKM ? 1 : 2)) * KS / 2, MI * NI * KS / 2>();
      }
    }
  }
  FD_STAMP(2);
  if constexpr (EPI == EPI_F32) {
    if (acs) {  // the 4 lane groups of a column hold disjoint k: fold them, lanes 0-15 store
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        float s = asum[i];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        const int m = m0 + wr * TM + i * 16 + lane;
        if (lane < 16 && m < p.M) {
          if (p.acol_p) {  // the bias's Adam step (fused epilogues never accumulate)
            float ss, inv;
            adam_bias_corr(p.adam.step, p.adam.lr, p.adam.b1, p.adam.b2, ss, inv);
            float pb = p.acol_p[m], mb = p.acol_m[m], vb = p.acol_v[m];
            adam_elem(p.adam.lr, p.adam.b1, p.adam.b2, p.adam.eps, p.adam.wd, p.adam.decoupled, pb, s, mb, vb, ss,
                      inv);
            p.acol_p[m] = pb;
            p.acol_m[m] = mb;
            p.acol_v[m] = vb;
            if (p.acol_sh) p.acol_sh[m] = (uint16_t)f2bf(pb);
          } else {
            p.acol[m] = p.accumulate ? p.acol[m] + s : s;
          }
        }
      }
    }
  }
  if constexpr (EpiTraits<EPI, BM, BN>::DIRECT) {
    // fp32 tile too large for LDS: finish it one wave-row band (TM rows) at a time through the
    // staged row-chunk epilogue (coalesced 16-byte rows for the gradient / Adam streams)
    constexpr int LDC = BN * 4 + 16;
    if (p.diag & 4) return;
#pragma unroll 1
    for (int band = 0; band < WM; ++band) {
      __syncthreads();  // ring slots (first band) / the previous band's staging are free
      if (wr == band) {
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int r = i * 16 + (lane & 15);
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            const int c = wc * TN + j * 16 + 4 * (lane >> 4);
            *reinterpret_cast<float4*>(smem + r * LDC + c * 4) =
                make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
          }
        }
      }
      __syncthreads();
      f32_epilogue<TM, BN, 64 * NW>(p, smem, LDC, m0 + band * TM, n0, tid);
    }
  } else if constexpr (EpiTraits<EPI, BM, BN>::LN2) {
    static_assert((BM == 128 || BM == 256) && BN == 128 && WM == 4 && TN == 64, "two-K-half LayerNorm tile");
    constexpr bool BWD2 = EPI == EPI_LN2_BWD;
    const int s = p.ln2_half, tn_ln = 2 * tn + s, pair = tm * (p.N / BN) + tn;
    const uint32_t tag =
        (uint32_t)__hip_atomic_load(p.ln.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * FD_LN_XSITES + p.ln.xsite + 1u;
    ln2_send<MI, NI>(p, acc, pair, s, wr, wc, lane, tag);  // (its barrier: no wave still reads a ring slot)
    // this block's LayerNorm operands in flight while the partner's partial arrives (issued before
    // the send instead, their latency joins the senders' drain and delays the flag: 1.619 vs
    // 1.606 ms/step, profiles/r5_rejected_ab.txt)
    const auto pre = ln_prefetch<BM, 64, BWD2, 64 * NW>(p, tm, tn_ln, tid);
    ln2_recv<MI, NI>(p, acc, pair, s, wc, wr, lane, tag);
    if (wc == s) ln_park<BM, 64, TM, TN, BWD2>(p, acc, smem, tn_ln * 64, wr, 0, lane);
    ln_finish<BM, 64, BWD2, 64 * NW>(p, smem, tm, tn_ln, lane, tid, pre);
  } else if constexpr (EpiTraits<EPI, BM, BN>::LN) {
    if (LNPF && lnpf) {
      wait_vm<0>();     // this wave's epilogue DMAs have landed ...
      __syncthreads();  // ... and every wave's; no wave still reads a ring slot
      const auto pre = ln_from_lds<BM, BN, EPI == EPI_LN_BWD, 64 * NW>(p, tm, tn, tid, smem);
      // (the tile is parked behind the prefetched operands: slots 2.. of the ring)
      ln_epilogue<BM, BN, TM, TN, EPI == EPI_LN_BWD, 64 * NW>(p, acc, smem + 2 * BUF, tm, tn, wr, wc, lane, tid, pre);
    } else {
      const auto pre = ln_prefetch<BM, BN, EPI == EPI_LN_BWD, 64 * NW>(p, tm, tn, tid);
      __syncthreads();  // no wave still reads a ring slot
      ln_epilogue<BM, BN, TM, TN, EPI == EPI_LN_BWD, 64 * NW>(p, acc, smem, tm, tn, wr, wc, lane, tid, pre);
    }
  } else {
    // every DMA has been waited for (the last iteration waits vmcnt(0)); after this
    // barrier no wave still reads a ring slot, so the epilogue may reuse the LDS.
    __syncthreads();
    staged_epilogue<BM, BN, TM, TN, EPI, 64 * NW, WT>(p, acc, smem, m0, n0, wr, wc, lane, tid);
  }
}

// bid = the tile's index within p, walked in group-M order
template <int BM, int BN, bool AK, bool BKM, int EPI, int WM, int WN, int S, int BK = BKT>
DEV void gemm_tile(const GemmParams& p, int bid, char* smem) {
  int tm, tn;
  tile_coords(bid, (p.M + BM - 1) / BM, p.N / BN, p.group_m, tm, tn);
  gemm_tile_at<BM, BN, AK, BKM, EPI, WM, WN, S, BK>(p, tm, tn, smem);
}

template <int BM, int BN, bool AK, bool BKM, int EPI, int WM, int WN, int S>
__global__ __launch_bounds__(64 * WM * WN, 2) void gemm_kernel(GemmParams p0, GemmGroup grp) {
  using G = GemmCfg<BM, BN, AK, BKM, EPI, WM, WN, S>;
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  FD_STAMP(0);
  stamp_hwid();
  int bid = xcd_remap(blockIdx.x, grp.ntiles);
  const bool second = bid >= grp.ntiles0;  // block-uniform
  const GemmParams& p = second ? grp.q : p0;
  if (second) bid -= grp.ntiles0;
  gemm_tile<BM, BN, AK, BKM, EPI, WM, WN, S>(p, bid, smem);
#if FD_GEMM_STAMPS
  __syncthreads();
  FD_STAMP(5);
#endif
}

// ---------------------------------------------------------------- QKV projection + attention forward
// One launch instead of two per block: blocks [0, ntiles) are the QKV GEMM's
// 128 x 192 tiles (cfg 6, bias epilogue), blocks after them the S <= 128 attention forward's
// (sequence, head) items (attn_fwd_s128_body, attn_s128.h).  A tile's bf16 output goes out with
// write-through (sc1) stores that every thread drains; then ONE lane stores the tile's {tag, 1}
// granule (agent-scope relaxed atomic, no fence: gfx950's release fence would write back the whole
// L2).  An attention item polls the granules of the tiles holding its rows' Q, K and V columns
// (<= 2 row blocks x 3 column tiles), then stages them with sc1 loads -- the LayerNorm exchange's
// hand-off (ln2_send / ln2_recv).  The tag is the exchange's: epoch * FD_LN_XSITES + xsite + 1, so
// granules of earlier launches never match.  Progress: a GEMM tile never waits, and every tile has
// a lower block index than every attention item, so the items wait only on tiles that were
// dispatched before them.  The poll is bounded (0.25 s; err |= 4, fatal on the host).
struct QkvAttnSync {
  uint64_t* flags;  // [ntiles] tile granules (the LayerNorm state's tail: zeroed at a tag wrap)
  const int* cnt;   // exchange epoch (advanced once per model forward)
  int* err;
  int xsite;
  int ntiles, tiles_n;
};
constexpr int QA_BM = 128, QA_BN = 192, QA_NW = 8;
using QaCfg = GemmCfg<QA_BM, QA_BN, true, true, EPI_BIAS, 2, 4, 2>;
static_assert(QaCfg::VALID && QaCfg::NW == QA_NW && QaCfg::SMEM >= ATT_FWD_SMEM, "fused QKV + attention tile");

__global__ __launch_bounds__(64 * QA_NW, 2) void gemm_attn_fwd_kernel(GemmParams p, AttnArgs a, QkvAttnSync q) {
  __shared__ __attribute__((aligned(1024))) char smem[QaCfg::SMEM];
  const uint32_t tag =
      (uint32_t)__hip_atomic_load(q.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * FD_LN_XSITES + q.xsite + 1u;
  if ((int)blockIdx.x < q.ntiles) {
    FD_STAMP(0);
    stamp_hwid();
    int tm, tn;
    tile_coords(xcd_remap(blockIdx.x, q.ntiles), (p.M + QA_BM - 1) / QA_BM, q.tiles_n, p.group_m, tm, tn);
    gemm_tile_at<QA_BM, QA_BN, true, true, EPI_BIAS, 2, 4, 2, BKT, true>(p, tm, tn, smem);
    __syncthreads();  // every thread's write-through stores have completed
    if (threadIdx.x == 0)
      __hip_atomic_store(q.flags + tm * q.tiles_n + tn, ((uint64_t)tag << 32) | 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  const int item = (int)blockIdx.x - q.ntiles, b = item / a.H, h = item - b * a.H;
  if (b < a.B) {  // (the filler item b == B reads no projection)
    int tok0, len;
    seq_span(a, b, tok0, len);
    if (len > 0 && threadIdx.x < 64) {
      const int lane = threadIdx.x, D = a.H * DH;
      const int tm0 = tok0 / QA_BM, nf = ((tok0 + len - 1) / QA_BM - tm0 + 1) * 3;
      uint64_t* fp = nullptr;
      if (lane < nf) fp = q.flags + (tm0 + lane / 3) * q.tiles_n + ((lane % 3) * D + h * DH) / QA_BN;
      const uint64_t t0 = wall_clock64();
      for (;;) {
        const bool ok = fp == nullptr || (uint32_t)(ld_gran(fp) >> 32) == tag;
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > 25000000ull) {  // 0.25 s: never in a healthy launch
          if (lane == 0) __hip_atomic_fetch_or(q.err, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();  // (no load of the body is issued before the poll matched)
  }
  attn_fwd_s128_body<QA_NW, 1>(a, b, h, 0, smem);
}

// ---------------------------------------------------------------- per-(sequence, head) QKV + attention
// Mode 2 of the fused QKV + attention forward: one block per (sequence, head) computes that head's
// Q, K and V columns of the sequence's rows itself -- a 128 x 192 projection tile whose A rows start
// at the sequence's first packed row and whose B rows are W's rows h 64.., D + h 64.., 2 D + h 64..
// -- and parks it (bias added, bf16: the values the separate GEMM stores) straight into the
// attention's swizzled LDS images, so the attention needs no global round trip and no hand-off.
// The K loop is gemm_tile_at's (same MFMA chain per element, so qkv is bitwise the GEMM's); the A
// rows past the sequence's live 16-row sub-tiles are neither loaded (their DMA pieces are skipped:
// the loop is bound by the per-CU fill rate) nor multiplied (their rows are never stored).  The
// sequence's qkv rows still go out (the backward reads them); filler rows past cu[B] are zeroed.
// Blocks walk the (sequence, head) items sequence-major after the XCD remap (an XCD's blocks share
// their sequences' x rows in its L2).  25.3 vs 15.6 + 10.2 us per layer for the two launches.
struct SeqQkvArgs {
  const bf16_t* x;   // [M][K]
  const bf16_t* w;   // [3 D][K]
  const float* bias; // [3 D]
  int M, K;
  int seq_major;     // logical item order: 0 head-major (an XCD walks ~1.5 heads), 1 sequence-major
};
using SaA = Operand<128, true, 8>;
using SaB = Operand<192, true, 8>;
constexpr int SA_S = 2, SA_BUF = SaA::BYTES + SaB::BYTES;
static_assert(SA_S * SA_BUF >= ATT_FWD_SMEM_Q, "the attention images fit the projection ring");

// The sequence's A rows only: the 1 KiB DMA pieces (8 rows each) of rows past the live 16-row
// sub-tiles are skipped (their accumulators stay 0; the ring waits vmcnt(0), so no count to keep)
DEV void sa_stage_a(const bf16_t* x, int ld, int row0, int k0, int lim, int rows_live, char* lds, int wid,
                    int lane) {
  const char* sbase = reinterpret_cast<const char*>(x + k0);
#pragma unroll
  for (int i = 0; i < SaA::PER_WAVE; ++i) {
    const int piece = wid * SaA::PER_WAVE + i;
    if (piece * 8 >= rows_live) continue;  // (wave-uniform)
    const int pos = piece * 64 + lane;
    const int r = pos >> 3, c = (pos & 7) ^ ksw(r);
    const int gr = min(row0 + r, lim - 1);
    glds16(sbase + (uint32_t)(gr * ld + c * 8) * 2u, lds + piece * 1024);
  }
}

// head h's Q, K, V weight rows as one 192-row K-major B tile (Operand::stage with a row map)
DEV void sa_stage_b(const bf16_t* w, int ld, int D, int h, int k0, char* lds, int wid, int lane) {
  const char* sbase = reinterpret_cast<const char*>(w + k0);
#pragma unroll
  for (int i = 0; i < SaB::PER_WAVE; ++i) {
    const int piece = wid * SaB::PER_WAVE + i;
    const int pos = piece * 64 + lane;
    const int r = pos >> 3, c = (pos & 7) ^ ksw(r);
    const int gr = h * DH + (r >> 6) * D + (r & 63);
    glds16(sbase + (uint32_t)(gr * ld + c * 8) * 2u, lds + piece * 1024);
  }
}

DEV void sa_project(const SeqQkvArgs& g, const AttnArgs& a, int tok0, int len, int h, char* smem) {
  constexpr int WN = 4, TM = 64, TN = 48, MI = TM / 16, NI = TN / 16;
  constexpr int L = SaA::PER_WAVE + SaB::PER_WAVE;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;
  const int D = a.H * DH, nk = g.K / BKT;
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // live 16-row sub-tiles of this wave's 64 rows (wave-uniform), and the tile's live rows
  const int rem = len - wr * TM, live = rem <= 0 ? 0 : min(MI, (rem + 15) >> 4);
  const int rows_live = min(128, (len + 15) & ~15);
  auto issue = [&](int t) {
    char* b = smem + (t % SA_S) * SA_BUF;
    sa_stage_a(g.x, g.K, tok0, t * BKT, g.M, rows_live, b, wid, lane);
    sa_stage_b(g.w, g.K, D, h, t * BKT, b + SaA::BYTES, wid, lane);
  };
  issue(0);
  for (int kt = 0; kt < nk; ++kt) {
    wait_tiles<L, 0>(0);  // tile kt has landed (the ring holds one tile in flight)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + 1 < nk) issue(kt + 1);  // into the slot everyone finished reading
    const char* cur = smem + (kt % SA_S) * SA_BUF;
    if (live > 0) {  // (the MFMAs of dead sub-tiles are skipped)
      bf16x8 a0[MI], b0[NI], a1[MI], b1[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) a0[i] = SaA::frag(cur, wr * TM + i * 16, 0, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) b0[j] = SaB::frag(cur + SaA::BYTES, wc * TN + j * 16, 0, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i) a1[i] = SaA::frag(cur, wr * TM + i * 16, 1, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) b1[j] = SaB::frag(cur + SaA::BYTES, wc * TN + j * 16, 1, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
        if (i < live)
#pragma unroll
          for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(b0[j], a0[i], acc[i][j]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
        if (i < live)
#pragma unroll
          for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(b1[j], a1[i], acc[i][j]);
    }
  }
  __syncthreads();  // no wave still reads a ring slot (the last wait drained every DMA)
  // accumulators + bias -> bf16 -> the attention's Q / K / V images (attn_fwd_s128_body MODE 2)
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int c = wc * TN + j * 16 + 4 * (lane >> 4), sec = c >> 6, cc = c & 63;
    const float4 bv = *reinterpret_cast<const float4*>(g.bias + sec * D + h * DH + cc);
    char* img = sec == 0 ? smem + ATT_FWD_SMEM : smem + (sec - 1) * 2 * 8192;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int r = wr * TM + i * 16 + (lane & 15);
      const uint2 v = make_uint2(pack_bf2(acc[i][j][0] + bv.x, acc[i][j][1] + bv.y),
                                 pack_bf2(acc[i][j][2] + bv.z, acc[i][j][3] + bv.w));
      *reinterpret_cast<uint2*>(img + (r >> 6) * 8192 + tile_off(r & 63, cc >> 3) + (cc & 7) * 2) = v;
    }
  }
  __syncthreads();
  // the sequence's projection rows out (the backward reads qkv)
  bf16_t* qkv = const_cast<bf16_t*>(a.qkv);
  const int ld3 = 3 * D;
#pragma unroll 2
  for (int id = tid; id < 128 * 24; id += 512) {
    const int r = id / 24, ch = id - r * 24, sec = ch >> 3, c8 = ch & 7;
    if (r < len) {
      const char* img = sec == 0 ? smem + ATT_FWD_SMEM : smem + (sec - 1) * 2 * 8192;
      *reinterpret_cast<uint4*>(qkv + (size_t)(tok0 + r) * ld3 + sec * D + h * DH + c8 * 8) =
          *reinterpret_cast<const uint4*>(img + (r >> 6) * 8192 + tile_off(r & 63, c8));
    }
  }
}

__global__ __launch_bounds__(512, 2) void seq_attn_fwd_kernel(SeqQkvArgs g, AttnArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[SA_S * SA_BUF];
  const int nb = a.B + (a.cu ? 1 : 0);
  // head-major logical order: after the XCD remap one XCD walks ~1.5 heads (their weight slices
  // stay in its L2) over every sequence
  const int item = xcd_remap(blockIdx.x, nb * a.H);
  const int h = g.seq_major ? item % a.H : item / nb, b = g.seq_major ? item / a.H : item - h * nb;
  if (b < a.B) {
    int tok0, len;
    seq_span(a, b, tok0, len);
    if (len > 0 && len <= 128) sa_project(g, a, tok0, len, h, smem);  // (longer: skipped by the body too)
  } else {  // filler rows of qkv: finite zeros (the separate GEMM's rows there are never read)
    zero_filler_at(a, const_cast<bf16_t*>(a.qkv), 3 * a.H * DH, 3, h, 0, 1);
  }
  attn_fwd_s128_body<8, 2>(a, b, h, 0, smem);
}

// ---------------------------------------------------------------- out-projection dX + attention backward
// The attention backward of a (sequence, head) computes its own dO -- that head's 64 columns of the
// out-projection's input gradient dctx = dy W (dy = the out-projection's output gradient [T][D],
// W = its weight [D][D] as the MN-major B operand, exactly linear_dx's NN GEMM) -- for the sequence's
// rows, straight into the backward's swizzled dO image: no dctx round trip through HBM and no launch
// of its own.  The Q / K / V loads of the backward are in flight across the K loop, whose 3-slot ring
// (two tiles in flight, counted waits) borrows the image region.  Same per-element MFMA chain as the cfg-24 NN GEMM (128 x 64,
// 4 x 2 waves), so dO -- and with it every gradient -- is bitwise the two-launch path's.  Rows past
// the sequence's live 16-row sub-tiles are neither loaded nor multiplied (dO 0 there: rows whose
// probabilities are exactly 0).
struct OProjArgs {
  const bf16_t* dy;  // [M][K] (the compact [CLS] form: [Bp][K], row b = sequence b's)
  const bf16_t* w;   // [K][D]: W itself (MN-major B)
  int M, K;
  int ksplit;        // K tiles per split: the split-K GEMM's partial chains, summed in split order
                     // (its slab reduce), when dy is the pruned block's M <= 64 compact rows
  int order;         // block -> (sequence, head): 1 XCD-remapped sequence-major, 0 launch order
};
using OpA = Operand<128, true, 8>;
using OpB = Operand<64, false, 8>;
constexpr int OP_BUF = OpA::BYTES + OpB::BYTES, OP_S = 3;
// the 3-slot ring spans the Q / K / V / dO images and the row tables after them: all written after it
constexpr int OP_SMEM = OP_S * OP_BUF > ATT_BWD_SMEM ? OP_S * OP_BUF : ATT_BWD_SMEM;
static_assert(OP_SMEM <= 80 * 1024, "two blocks per CU");

// rows [tok0, tok0 + len) of dy -> dO image rows [0, len); image rows >= keep are written as zeros
// (the compact form: one row, the others' dO 0 like stage_cls_rows)
DEV void op_project(const OProjArgs& pj, const AttnArgs& a, int tok0, int len, int h, char* smem, int keep = 128) {
  constexpr int WN = 2, TM = 32, TN = 32, MI = TM / 16, NI = TN / 16;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;
  const int D = a.H * DH, nk = pj.K / BKT;
  const int rem = len - wr * TM, live = rem <= 0 ? 0 : min(MI, (rem + 15) >> 4);
  const int rows_live = min(128, (len + 15) & ~15);
  f32x4 acc[MI][NI], tot[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = tot[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool split = pj.ksplit < nk;  // (uniform)
  // this wave's DMA ops per K tile (its A pieces of live rows + one B piece): the counted ring wait
  const int ops = (wid * OpA::PER_WAVE * 8 < rows_live ? 1 : 0) + ((wid * OpA::PER_WAVE + 1) * 8 < rows_live ? 1 : 0) +
                  OpB::PER_WAVE;
  static_assert(OpA::PER_WAVE == 2, "ops count");
  auto issue = [&](int t) {
    char* sl = smem + (t % OP_S) * OP_BUF;
    const char* abase = reinterpret_cast<const char*>(pj.dy + t * BKT);
#pragma unroll
    for (int i = 0; i < OpA::PER_WAVE; ++i) {  // the sequence's live A rows only (8 rows per piece)
      const int piece = wid * OpA::PER_WAVE + i;
      if (piece * 8 >= rows_live) continue;
      const int pos = piece * 64 + lane;
      const int r = pos >> 3, c = (pos & 7) ^ ksw(r);
      glds16(abase + (uint32_t)(min(tok0 + r, pj.M - 1) * pj.K + c * 8) * 2u, sl + piece * 1024);
    }
    OpB::stage(pj.w, D, h * DH, t * BKT, D, sl + OpA::BYTES, wid, lane);
  };
  issue(0);
  if (nk > 1) issue(1);
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt landed; tile kt + 1 (if any) stays in flight
    if (kt + 1 < nk) wait_ops(ops);
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // ... in every wave; everyone also finished reading tile kt - 1's slot
    asm volatile("" ::: "memory");
    if (kt + 2 < nk) issue(kt + 2);
    const char* cur = smem + (kt % OP_S) * OP_BUF;
    if (live > 0) {
      bf16x8 a0[MI], b0[NI], a1[MI], b1[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) a0[i] = OpA::frag(cur, wr * TM + i * 16, 0, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) b0[j] = OpB::frag(cur + OpA::BYTES, wc * TN + j * 16, 0, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i) a1[i] = OpA::frag(cur, wr * TM + i * 16, 1, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) b1[j] = OpB::frag(cur + OpA::BYTES, wc * TN + j * 16, 1, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
        if (i < live)
#pragma unroll
          for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(b0[j], a0[i], acc[i][j]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
        if (i < live)
#pragma unroll
          for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(b1[j], a1[i], acc[i][j]);
    }
    if (split && kt % pj.ksplit == pj.ksplit - 1) {  // a split's partial: added in split order, then restart
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          tot[i][j] = tot[i][j] + acc[i][j];
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
  }
  if (split) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = tot[i][j];
  }
  __syncthreads();  // every wave is done with the ring (the Q / K / V images go there next)
  char* os = smem + 6 * 8192;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int r = wr * TM + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int c = wc * TN + j * 16 + 4 * (lane >> 4);
      *reinterpret_cast<uint2*>(os + (r >> 6) * 8192 + tile_off(r & 63, c >> 3) + (c & 7) * 2) =
          r < keep ? make_uint2(pack_bf2(acc[i][j][0], acc[i][j][1]), pack_bf2(acc[i][j][2], acc[i][j][3]))
                   : make_uint2(0u, 0u);
    }
  }
}

__global__ __launch_bounds__(512) void attn_bwd_proj_kernel(AttnArgs a, OProjArgs pj) {
  __shared__ __attribute__((aligned(1024))) char smem[OP_SMEM];
  // 1-D grid, XCD remap: sequence-major (one XCD's blocks share their sequences' dy rows in its L2),
  // or the hardware (head, sequence) order of the 3-D grid (pj.order 0)
  int b, h;
  if (pj.order) {
    const int item = xcd_remap(blockIdx.x, gridDim.x);
    h = item % a.H;
    b = item / a.H;
  } else {
    h = blockIdx.x % a.H;
    b = blockIdx.x / a.H;
  }
  // compact [CLS] form (a.dres): dO row 0 = dy row b, every other row 0
  auto proj = [&](int tok0, int len) {
    if (a.dres) op_project(pj, a, b, 1, h, smem, 1);
    else op_project(pj, a, tok0, len, h, smem);
  };
  attn_bwd_s128_body<2>(a, b, h, smem, proj);
}

// LayerNorm-fused NT GEMM (EPI_LN / EPI_LN_BWD): the tiles of a row block are consecutive
// logical tiles (row-major tile order), so after the XCD remap they run on one XCD, in order.
// BKM = false: B is the weight W [K][N] itself (MN-major; the backward dX GEMMs without W^T).
template <int BM, int BN, int EPI, int WM, int WN, int S, bool BKM = true>
__global__ __launch_bounds__(64 * WM * WN, 2) void gemm_ln_kernel(GemmParams p) {
  using G = GemmCfg<BM, BN, true, BKM, EPI, WM, WN, S>;
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  FD_STAMP(0);
  stamp_hwid();
  const int tiles_n = p.N / BN;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  gemm_tile_at<BM, BN, true, BKM, EPI, WM, WN, S>(p, lid / tiles_n, lid % tiles_n, smem);
#if FD_GEMM_STAMPS
  __syncthreads();
  FD_STAMP(5);
#endif
}

// Two-K-half LayerNorm-fused GEMM (EPI_LN2 / EPI_LN2_BWD): block pair (lid / 2) owns the 128 x 128
// product tile pair, block lid % 2 its K half (A / B offset by that half; one K loop of K / 2).
// The pair's blocks are consecutive logical ids (one XCD after the remap); the row block's 12
// LayerNorm tiles stay consecutive.  One resident round (one 128 KiB block per CU).
// BM = 256 (256 x 128 product tiles, 256 x 64 LayerNorm tiles; 3 ring slots of 48 KiB): the
// larger batches (e.g. seq256 bs64, ~5.1 k packed rows) whose 128-row grid would exceed one round.
template <int EPI, bool BKM, int BM = 128>
__global__ __launch_bounds__(512, 1) void gemm_ln2_kernel(GemmParams p) {
  constexpr int S = BM == 128 ? 4 : 3;
  using G = GemmCfg<BM, 128, true, BKM, EPI, 4, 2, S>;
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  FD_STAMP(0);
  stamp_hwid();
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int pair = lid >> 1, s = lid & 1, tiles_n2 = p.N / 128;
  GemmParams q = p;
  const int kh = p.K / 2;
  q.A = p.A + (size_t)s * kh;
  q.B = BKM ? p.B + (size_t)s * kh : p.B + (size_t)s * kh * p.ldb;
  q.k_split = kh;
  q.ln2_half = s;
  gemm_tile_at<BM, 128, true, BKM, EPI, 4, 2, S>(q, pair / tiles_n2, pair % tiles_n2, smem);
#if FD_GEMM_STAMPS
  __syncthreads();
  FD_STAMP(5);
#endif
}

// ---------------------------------------------------------------- all-layer weight gradients
// Every weight gradient of a backward pass in ONE launch, at the end of the backward
// (RunCtx.dw_batch, ops/functional.py): C_i[M_i][N_i] (+)= A_i^T B_i over the same token
// dimension K, for up to DWB_MAXP problems (4 per transformer block).  The per-layer grouped
// launches it replaces each fill the chip about once, so they need split-K (fp32 slabs + a
// reduce) and, with Adam fused into the epilogue, every tile reaches the optimizer traffic
// at the same moment (engine/optim.py: measured slower).  One launch over all layers has
// ~20 rounds of 128x64 tiles: no split-K (each tile runs the full K loop -- deterministic, no
// slabs), and tiles reach their epilogue -- plain store, or Adam (adam_epi4) -- staggered
// while other tiles are on the MFMAs.  Problems are laid out back to back in the logical
// tile order; after the XCD remap each XCD walks a contiguous range, i.e. 2-3 problems.
constexpr int DWB_MAXP = 32;
using DwProb = FdDwProb;  // adam_epi.h (shared with the host binding)
struct DwBatch {
  DwProb pr[DWB_MAXP];
  int n, K, ntiles, group_m;
  int diag;  // FD_GEMM_DIAG (profiling only)
  const int* step;
  float lr, b1, b2, eps, wd;
  int decoupled;
  FdAdamRest rest;  // rest.p != nullptr: blocks [ntiles, ntiles + rest blocks) finish the optimizer step
  // Mixed schedule (fd_gemm_dw_batch plan_dwb_mix; mixed != 0): problems are ordered in three classes
  // -- [long 256 x 256 | long 256 x 128 (half) | short-K 256 x 256] -- and each class is dealt to the
  // 8 XCDs in contiguous ranges of cls_pad[c] blocks per XCD (padding blocks return at once), so every
  // XCD runs its full-size long tiles first, then its share of the half tiles and short tiles in the
  // rounds the long tiles leave partly idle.
  int mixed;
  int cls_tiles[3], cls_off[3], cls_pad[3];
};

// The mixed schedule's half tiles: 256 x 128 on the same 8 waves (4 x 2, 64 x 64 per wave).  Every
// output element runs the same K-step / MFMA chain as in a 256 x 256 tile and the same f32_epilogue
// (Adam) arithmetic, so a problem's gradient and optimizer step are bitwise those of the full tiles.
constexpr int DWB_HBM = 256, DWB_HBN = 128, DWB_HWM = 4, DWB_HWN = 2;

// One tile of the batch: logical tile id lid -> (problem, tile) -> K loop + epilogue.
template <int BM, int BN, int WM, int WN, int S, int BK, bool MIX = false>
DEV void dwb_tile(const DwBatch& bt, int lid, char* smem) {
  int i = 0;
  while (i + 1 < bt.n && lid >= bt.pr[i + 1].tile0) ++i;  // block-uniform
  const DwProb& q = bt.pr[i];
  GemmParams p{};
  p.A = q.A; p.B = q.B; p.C = q.C;
  const int K = q.K > 0 ? q.K : bt.K;
  p.M = q.M; p.N = q.N; p.K = K;
  p.lda = q.M; p.ldb = q.N; p.ldc = q.N;
  p.k_split = K;
  p.group_m = bt.group_m;
  p.diag = bt.diag;
  p.out = q.C;
  p.accumulate = q.accumulate;
  p.acol = q.bias;
  if (q.p) {
    p.adam.p = q.p; p.adam.m = q.m; p.adam.v = q.v; p.adam.sh = q.sh; p.adam.step = bt.step;
    p.adam.lr = bt.lr; p.adam.b1 = bt.b1; p.adam.b2 = bt.b2; p.adam.eps = bt.eps; p.adam.wd = bt.wd;
    p.adam.decoupled = bt.decoupled;
    if (q.bias && bt.rest.p) {  // the qkv bias's state lies at its gradient's arena offset
      const ptrdiff_t off = q.bias - bt.rest.g;
      p.acol_p = bt.rest.p + off; p.acol_m = bt.rest.m + off; p.acol_v = bt.rest.v + off;
      p.acol_sh = bt.rest.sh ? bt.rest.sh + off : nullptr;
    }
  }
  if constexpr (MIX) {
    if (q.half) {  // block-uniform
      gemm_tile<DWB_HBM, DWB_HBN, false, false, EPI_F32, DWB_HWM, DWB_HWN, S, BK>(p, lid - q.tile0, smem);
      return;
    }
  }
  gemm_tile<BM, BN, false, false, EPI_F32, WM, WN, S, BK>(p, lid - q.tile0, smem);
}

// Mixed schedule: tile block b (past the rest blocks, whose count is a multiple of 8, so b % 8 is
// the block's XCD) -> logical tile id, or -1 for a padding block.
DEV int dwb_mixed_lid(const DwBatch& bt, int b) {
  const int x = b % 8;
  int j = b / 8, c = 0;
  while (c < 2 && j >= bt.cls_pad[c]) {
    j -= bt.cls_pad[c];
    ++c;
  }
  if (j >= bt.cls_pad[c]) return -1;
  const int t = x * bt.cls_pad[c] + j;
  return t < bt.cls_tiles[c] ? bt.cls_off[c] + t : -1;
}

// Blocks past the tiles: the rest of the optimizer step (FdAdamRest), dispatched after every tile,
// i.e. on the CUs the launch's last, partial round of tiles leaves idle.  The first flat_blocks
// walk the run table (adam_kernel<true, true>'s element body), the others take 64-row flag chunks
// of the word table per wave (adam_rows_kernel's row body) -- the same arithmetic, bitwise.
constexpr int DWB_RUNS_LDS = 4096;  // run-table entries (3 per run) staged in LDS by the flat rest blocks
template <int NT>
DEV void dwb_rest(const DwBatch& bt, int rb, char* smem) {
  const FdAdamRest& r = bt.rest;
  float ss, inv;
  adam_bias_corr(bt.step, bt.lr, bt.b1, bt.b2, ss, inv);
  AdamArgs a{};
  a.step = bt.step; a.lr = bt.lr; a.b1 = bt.b1; a.b2 = bt.b2; a.eps = bt.eps;
  if (rb < r.flat_blocks) {
    a.p = r.p; a.g = r.g; a.m = r.m; a.v = r.v; a.shadow = reinterpret_cast<bf16_t*>(r.sh);
    a.wd = bt.wd; a.decoupled = bt.decoupled;
    a.runs = r.runs; a.nruns = r.nruns; a.n4 = r.n4;
    // adam_flat4's element body (the same arithmetic, bitwise), U float4 per thread at once: the
    // run lookups binary-search an LDS copy of the run table, and every load of the U elements is
    // issued before their stores (in turn each lookup chain and each load would wait for the
    // previous element's stores; 1.625 vs 1.629 ms/step, profiles/r5_ab_rest_adam_batched.txt)
    if (r.runs && 3 * r.nruns <= DWB_RUNS_LDS) {
      long long* rl = reinterpret_cast<long long*>(smem);
      for (int i = threadIdx.x; i < 3 * r.nruns; i += NT) rl[i] = r.runs[i];
      __syncthreads();
      a.runs = rl;
    }
    constexpr int U = 4;
    const long long stride = (long long)r.flat_blocks * NT;
    for (long long v0 = (long long)rb * NT + threadIdx.x; v0 < r.n4; v0 += U * stride) {
      long long idx[U];
      float4 p4[U], g4[U], m4[U], v4[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long vi = min(v0 + u * stride, r.n4 - 1);
        idx[u] = a.runs ? run_index(a.runs, a.nruns, vi) : vi;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        p4[u] = ld_nt(reinterpret_cast<const float4*>(a.p) + idx[u]);
        g4[u] = ld_nt(reinterpret_cast<const float4*>(a.g) + idx[u]);
        m4[u] = ld_nt(reinterpret_cast<const float4*>(a.m) + idx[u]);
        v4[u] = ld_nt(reinterpret_cast<const float4*>(a.v) + idx[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (v0 + u * stride >= r.n4) continue;
        const long long i = idx[u];
        float pp[4] = {p4[u].x, p4[u].y, p4[u].z, p4[u].w}, gg[4] = {g4[u].x, g4[u].y, g4[u].z, g4[u].w};
        float mm[4] = {m4[u].x, m4[u].y, m4[u].z, m4[u].w}, vv[4] = {v4[u].x, v4[u].y, v4[u].z, v4[u].w};
        adam_math4(a, pp, gg, mm, vv, ss, inv);
        st_nt(reinterpret_cast<float4*>(a.p) + i, make_float4(pp[0], pp[1], pp[2], pp[3]));
        st_nt(reinterpret_cast<float4*>(a.m) + i, make_float4(mm[0], mm[1], mm[2], mm[3]));
        st_nt(reinterpret_cast<float4*>(a.v) + i, make_float4(vv[0], vv[1], vv[2], vv[3]));
        if (a.shadow)
          reinterpret_cast<uint2*>(a.shadow)[i] = make_uint2(pack_bf2(pp[0], pp[1]), pack_bf2(pp[2], pp[3]));
      }
    }
    return;
  }
  if (!r.ever) return;
  a.p = r.p + r.woff; a.g = r.g + r.woff; a.m = r.m + r.woff; a.v = r.v + r.woff;
  a.shadow = r.sh ? reinterpret_cast<bf16_t*>(r.sh) + r.woff : nullptr;
  a.wd = 0.f; a.decoupled = 0;
  a.touched = r.ever; a.now = r.now;
  const int lane = threadIdx.x & 63;
  const int nwaves = r.row_blocks * (NT / 64);
  for (int r0 = ((rb - r.flat_blocks) * (NT / 64) + (int)(threadIdx.x >> 6)) * 16; r0 < r.wrows; r0 += nwaves * 16)
    adam_rows16(a, r0, r.wrows, r.wrow4, lane, ss, inv);
}

template <int BM, int BN, int WM, int WN, int S, int BK, bool MIX>
constexpr int dwb_smem() {
  using G = GemmCfg<BM, BN, false, false, EPI_F32, WM, WN, S, BK>;
  using H = GemmCfg<DWB_HBM, DWB_HBN, false, false, EPI_F32, DWB_HWM, DWB_HWN, S, BK>;
  return MIX && H::SMEM > G::SMEM ? H::SMEM : G::SMEM;
}

template <int BM, int BN, int WM, int WN, int S, int BK = BKT, bool MIX = false>
__global__ __launch_bounds__(64 * WM * WN, 2) void gemm_dw_batch_kernel(DwBatch bt) {
  constexpr int SMEM = dwb_smem<BM, BN, WM, WN, S, BK, MIX>();
  static_assert(SMEM <= LDS_MAX, "LDS");
  static_assert(!MIX || (BM == DWB_HBM && WM * WN == DWB_HWM * DWB_HWN), "mixed tiles share the block shape");
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  // the rest blocks lead the grid (their HBM stream beside the first round's K loops, while the
  // memory is otherwise idle) or follow the tiles (on the CUs the last, partial round leaves idle);
  // a leading group is a multiple of 8 blocks, so every tile keeps its XCD under xcd_remap
  const int nrest = bt.rest.flat_blocks + bt.rest.row_blocks;
  int bid = blockIdx.x;
  if (bt.rest.first) {
    if (bid < nrest) {  // block-uniform
      dwb_rest<64 * WM * WN>(bt, bid, smem);
      return;
    }
    bid -= nrest;
  } else {
    const int nblk = MIX && bt.mixed ? 8 * (bt.cls_pad[0] + bt.cls_pad[1] + bt.cls_pad[2]) : bt.ntiles;
    if (bid >= nblk) {
      dwb_rest<64 * WM * WN>(bt, bid - nblk, smem);
      return;
    }
  }
  if constexpr (MIX) {
    if (bt.mixed) {
      const int lid = dwb_mixed_lid(bt, bid);
      if (lid >= 0) dwb_tile<BM, BN, WM, WN, S, BK, true>(bt, lid, smem);
      return;
    }
  }
  dwb_tile<BM, BN, WM, WN, S, BK>(bt, xcd_remap(bid, bt.ntiles), smem);
}

// out[i] = (accumulate ? out[i] : 0) + sum_z slab[z][i]   (deterministic split-K reduce)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slabs, float* __restrict__ out,
                                                            long long n4, long long stride, int splits,
                                                            int accumulate) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float4 s = accumulate ? reinterpret_cast<float4*>(out)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int z = 0; z < splits; ++z) {
      const float4 v = reinterpret_cast<const float4*>(slabs + z * stride)[i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    reinterpret_cast<float4*>(out)[i] = s;
  }
}

// Deferred split-K reduces of a whole backward in one launch: job i owns blocks
// [start[i], start[i+1]) and reduces exactly like splitk_reduce_kernel (same z order).
constexpr int RED_MAXJ = 16;
struct ReduceJob {
  const float* slabs;
  float* out;
  long long n4, stride;
  int splits, accumulate;
};
struct ReduceBatch {
  ReduceJob j[RED_MAXJ];
  int start[RED_MAXJ + 1];
  int n;
};

__global__ __launch_bounds__(256) void splitk_reduce_batched_kernel(ReduceBatch rb) {
  int ji = 0;
  while (ji + 1 < rb.n && (int)blockIdx.x >= rb.start[ji + 1]) ++ji;
  const ReduceJob& jb = rb.j[ji];
  const int b0 = rb.start[ji], nb = rb.start[ji + 1] - b0;
  for (long long i = (blockIdx.x - b0) * 256ll + threadIdx.x; i < jb.n4; i += (long long)nb * 256) {
    float4 s = jb.accumulate ? reinterpret_cast<float4*>(jb.out)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int z = 0; z < jb.splits; ++z) {
      const float4 v = reinterpret_cast<const float4*>(jb.slabs + z * jb.stride)[i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    reinterpret_cast<float4*>(jb.out)[i] = s;
  }
}

// ---------------------------------------------------------------- configurations
// id: BM x BN, waves WM x WN, ring depth S   (LDS = max(S*(BM+BN)*128 B, epilogue))
//  0: 128 x  64, 2x2, S3      1: 128 x 128, 2x2, S2      2: 128 x  96, 2x2, S2 (K-major B)
//  3: 256 x 192, 4x2, S2      4: 256 x 128, 4x2, S3      5:  64 x 192, 1x4, S3
//  6: 128 x 192, 2x4, S2      7: 256 x  96, 4x1, S3 (K-major B)
//  8: 128 x  64, 2x2, S2      9: 128 x  96, 2x2, S3 (K-major B)
// 10: 128 x 128, 2x2, S3     11: 256 x 256, 2x4, S2     12: 256 x 128, 4x2, S2
// 13:  64 x  64, 2x2, S3     14:  64 x 128, 2x2, S3  (small tiles: 2-4 blocks/CU at N = 768)
// 15: 128 x  64, 2x2, S4     16: 128 x  64, 2x2, S5     17: 128 x 128, 2x2, S4  (deep rings:
//     more LDS-DMA bytes in flight per CU where the grid is one block per CU)
// 18: 128 x  64, 4x2, S3     19: 128 x  64, 4x2, S2     20: 128 x  64, 2x4, S3
// 21: 128 x 128, 4x2, S3  (8-wave blocks: two waves per SIMD where the grid is one block per CU)
// 22: 128 x  64, 2x2, S6     23:  64 x  64, 2x2, S6     24: 128 x  64, 4x2, S6  (two K tiles per barrier)
// Only the configurations some shape picks (pick_cfg / dw2_cfg / the LayerNorm-fused and all-layer
// dW launchers) are instantiated; the others were measured and lost (profiles/r1_gemm_cfg_sweep*,
// r1_ab_small_tiles.txt) and launch nothing (the caller falls back to cfg 0 / 8).  Removed after
// losing their A/B in the step: a ping-pong 8-wave variant (1.5-3x slower), a register-pipelined
// K loop (cfg 25-34; faster isolated, 1.911 vs 1.895-1.904 ms/step), a persistent per-XCD dW
// grid (cfg 41-44; neutral) and an in-kernel split-K fixup (2.89 vs 2.38 ms/step)
// (profiles/r2_ab_pipelined_gemm_persistent_dw.txt, r1_ab_fused_adam_fixup.txt).
constexpr int NCFG = 25;
struct CfgDesc { int bm, bn, wm, wn, s; };
constexpr CfgDesc CFGS[NCFG] = {{128, 64, 2, 2, 3}, {128, 128, 2, 2, 2}, {128, 96, 2, 2, 2}, {256, 192, 4, 2, 2},
                                {256, 128, 4, 2, 3}, {64, 192, 1, 4, 3}, {128, 192, 2, 4, 2}, {256, 96, 4, 1, 3},
                                {128, 64, 2, 2, 2},  {128, 96, 2, 2, 3}, {128, 128, 2, 2, 3}, {256, 256, 2, 4, 2},
                                {256, 128, 4, 2, 2}, {64, 64, 2, 2, 3},    {64, 128, 2, 2, 3},  {128, 64, 2, 2, 4},
                                {128, 64, 2, 2, 5},  {128, 128, 2, 2, 4}, {128, 64, 4, 2, 3},  {128, 64, 4, 2, 2},
                                {128, 64, 2, 4, 3},  {128, 128, 4, 2, 3}, {128, 64, 2, 2, 6},  {64, 64, 2, 2, 6},
                                {128, 64, 4, 2, 6}};

template <int BM, int BN, bool AK, bool BKM, int EPI, int WM, int WN, int S>
bool launch_cfg(const GemmParams& p, int splits, hipStream_t st, const GemmParams* q) {
  using G = GemmCfg<BM, BN, AK, BKM, EPI, WM, WN, S>;
  if constexpr (!G::VALID) {
    return false;
  } else {
    if (p.N % BN != 0) return false;
    GemmGroup grp{};
    grp.ntiles0 = ((p.M + BM - 1) / BM) * (p.N / BN);
    grp.ntiles = grp.ntiles0;
    if (q) {
      if (q->N % BN != 0 || q->M % BM != 0) return false;
      grp.q = *q;
      grp.ntiles += (q->M / BM) * (q->N / BN);
    }
    const dim3 grid(grp.ntiles, 1, splits);
    hipLaunchKernelGGL((gemm_kernel<BM, BN, AK, BKM, EPI, WM, WN, S>), grid, dim3(64 * WM * WN), 0, st, p, grp);
    return true;
  }
}

template <bool AK, bool BKM, int EPI>
bool launch_id(const GemmParams& p, int id, int splits, hipStream_t st, const GemmParams* q = nullptr) {
  switch (id) {
    case 0: return launch_cfg<128, 64, AK, BKM, EPI, 2, 2, 3>(p, splits, st, q);
    case 1: return launch_cfg<128, 128, AK, BKM, EPI, 2, 2, 2>(p, splits, st, q);
    case 3: return launch_cfg<256, 192, AK, BKM, EPI, 4, 2, 2>(p, splits, st, q);
    case 6: return launch_cfg<128, 192, AK, BKM, EPI, 2, 4, 2>(p, splits, st, q);
    case 8: return launch_cfg<128, 64, AK, BKM, EPI, 2, 2, 2>(p, splits, st, q);
    case 10: return launch_cfg<128, 128, AK, BKM, EPI, 2, 2, 3>(p, splits, st, q);
    case 11: return launch_cfg<256, 256, AK, BKM, EPI, 2, 4, 2>(p, splits, st, q);
    case 13: return launch_cfg<64, 64, AK, BKM, EPI, 2, 2, 3>(p, splits, st, q);
    case 18: return launch_cfg<128, 64, AK, BKM, EPI, 4, 2, 3>(p, splits, st, q);
    case 21: return launch_cfg<128, 128, AK, BKM, EPI, 4, 2, 3>(p, splits, st, q);
    case 24: return launch_cfg<128, 64, AK, BKM, EPI, 4, 2, 6>(p, splits, st, q);
  }
  return false;
}

// The configuration ids launch_id instantiates; an override naming any other id (measured and
// removed, see the table above) falls back to the automatic pick instead of failing the launch.
constexpr int INSTANTIATED[] = {0, 1, 3, 6, 8, 10, 11, 13, 18, 21, 24};
bool cfg_instantiated(int id) {
  for (int v : INSTANTIATED)
    if (v == id) return true;
  return false;
}

// Tuning overrides: per GEMM kind a forced config id / split count (-1 = auto),
// set from FD_GEMM_CFG_{NT,NN,TN} / FD_GEMM_SPLITS or at run time (fd_gemm_set_cfg).
int g_cfg_override[3] = {-2, -2, -2};
int g_ln_diag = -1;  // FD_GEMM_LN_DIAG / fd_gemm_ln_set_diag
int g_splits_override = -2;

int cfg_override(int kind) {
  if (g_cfg_override[kind] == -2) {
    const char* names[3] = {"FD_GEMM_CFG_NT", "FD_GEMM_CFG_NN", "FD_GEMM_CFG_TN"};
    const char* e = getenv(names[kind]);
    g_cfg_override[kind] = e && cfg_instantiated(atoi(e)) ? atoi(e) : -1;
  }
  return g_cfg_override[kind];
}
int splits_override() {
  if (g_splits_override == -2) {
    const char* e = getenv("FD_GEMM_SPLITS");
    g_splits_override = e ? atoi(e) : -1;
  }
  return g_splits_override;
}

long long tiles_of(int id, int M, int N) {
  const CfgDesc& c = CFGS[id];
  if (N % c.bn) return 0;
  return (long long)((M + c.bm - 1) / c.bm) * (N / c.bn);
}

// Default configuration per kind/shape, measured on MI355X at the DistilBERT
// shapes (M = 4096 tokens; scripts/gemm_sweep.py -> profiles/r1_gemm_cfg_sweep.txt).
// Occupancy wins over ring depth: the 2-3 blocks/CU configs (S2) beat the
// 1 block/CU S3 rings at every shape; 8-wave 256x192 / 128x192 only where they
// make one full round of tiles.
// M <= 64 (the pruned last block's [CLS] rows): 64 x 64 tiles -- a 128-row tile would be half
// empty, and a one-round grid's time is its per-tile K loop (FD_SMALLM_TILES=0: off)
bool smallm_tiles() {
  static const bool on = [] { const char* e = getenv("FD_SMALLM_TILES"); return !e || atoi(e) != 0; }();
  return on;
}

int pick_cfg(int kind, int M, int N, int K) {
  if (kind == 0 && M <= 64 && N % 64 == 0 && smallm_tiles()) return 13;
  if (kind == 0) {  // NT: forward (and any y = x B^T with a K-major B)
    // FFN1 forward / FFN2 dX (N = 3072): 256x192 fills the chip at M = 4096 (padded bs32),
    // 128x128 wins at the packed M ~ 2.7 k (21.5 vs 25.7 us; profiles/r1_gemm_cfg_sweep_T2688_packed.txt)
    // FD_GEMM_WIDE_CFG=<id>: configuration of the N >= 1536 NT GEMMs (QKV / FFN1 forward, FFN2 dX)
    static const int wide = [] { const char* e = getenv("FD_GEMM_WIDE_CFG"); return e ? atoi(e) : -1; }();
    if (cfg_instantiated(wide) && N >= 1536 && M >= 1024 && M <= 4096 && tiles_of(wide, M, N) > 0) return wide;
    // M >= 3584 (the distillation config's ~5.1 k packed rows, bs256 inference): 8-wave 128 x 192 tiles
    // -- 39.9 vs 49.4 us (256 x 192) for FFN1 at M = 5184, never slower from 4 k to 20 k rows
    // (profiles/r6_gemm_cfg_sweep_ffn_large_m.txt).  FD_GEMM_BIG_CFG=<id> overrides (3: the old pick).
    static const int big = [] { const char* e = getenv("FD_GEMM_BIG_CFG"); return e ? atoi(e) : 6; }();
    if (N % 192 == 0 && N >= 3072 && M >= 3584 && cfg_instantiated(big) && tiles_of(big, M, N) > 0) return big;
    if (N % 128 == 0 && N >= 3072 && M >= 2048) return 1;
    if (N % 192 == 0 && N >= 1536 && M >= 2048) return 6;
    // (N = 768 on 64 x 64 tiles -- 2-3 blocks per CU -- was faster in isolation but not in the
    // step, 2.370 vs 2.367 ms, profiles/r1_ab_small_tiles.txt: removed)
    // N = 768 at M <= 4 k (the packed / padded bs32 step): 8-wave 128 x 64 tiles with two K
    // tiles per barrier (cfg 24) -- one block per CU still gets two waves per SIMD, and the
    // loop pays half the barriers.  2.21-2.25 vs 2.28 ms/step in the model (3 A/B pairs,
    // profiles/r1_ab_narrow_cfg24.txt).  FD_GEMM_NARROW_CFG=<id> overrides (-1: the rule below).
    static const int narrow = [] { const char* e = getenv("FD_GEMM_NARROW_CFG"); return e ? atoi(e) : 24; }();
    if (cfg_instantiated(narrow) && N < 1536 && M >= 1024 && M <= 4096) return narrow;
    return K >= 2048 ? 0 : 8;
  }
  if (kind == 1) {  // NN dX (on the weight W itself: MN-major B through the transposing LDS reads)
    if (M <= 64 && N % 64 == 0 && smallm_tiles()) return 13;  // (as for NT: no half-empty 128-row tiles)
    // the NT rules above, measured equal per configuration (round 4, profiles/r4_ab_dx_layouts.txt:
    // the LayerNorm-fused dX reads W as fast as W^T on cfg 24)
    if (N % 192 == 0 && N >= 3072 && M >= 3584) return 3;
    if (N % 128 == 0 && N >= 3072 && M >= 2048) return 1;
    if (N % 192 == 0 && N >= 1536 && M >= 2048) return 6;
    static const int narrow = [] { const char* e = getenv("FD_GEMM_NARROW_CFG"); return e ? atoi(e) : 24; }();
    if (cfg_instantiated(narrow) && N < 1536 && M >= 1024 && M <= 4096) return narrow;
    return 8;
  }
  return (N % 128 == 0 && M > 1024 && M < 3072 && N < 3072) ? 1 : 8;  // TN dW
}

template <bool AK, bool BKM>
bool launch_epi(int epi, const GemmParams& p, int id, int splits, hipStream_t st) {
  switch (epi) {
    case EPI_BF16: return launch_id<AK, BKM, EPI_BF16>(p, id, splits, st);
    case EPI_BIAS: if constexpr (AK && BKM) return launch_id<AK, BKM, EPI_BIAS>(p, id, splits, st); break;
    case EPI_BIAS_GELU: if constexpr (AK && BKM) return launch_id<AK, BKM, EPI_BIAS_GELU>(p, id, splits, st); break;
    case EPI_GELU_BWD: if constexpr (AK) return launch_id<AK, BKM, EPI_GELU_BWD>(p, id, splits, st); break;
    case EPI_ADD: if constexpr (AK) return launch_id<AK, BKM, EPI_ADD>(p, id, splits, st); break;
    case EPI_F32: if constexpr (BKM == AK) return launch_id<AK, BKM, EPI_F32>(p, id, splits, st); break;
  }
  return false;
}

// Launch the weight-gradient GEMM(s) ps[0..nprob) (ps[i].C = final fp32 gradient, k_split
// unset) with `splits` K splits: direct (one split) or fp32 slabs + a deterministic reduce.
// adams[i].p != nullptr fuses Adam into the epilogue (one split only).
int dw_launch(GemmParams* ps, int nprob, int id, int splits, int K, float* workspace, long long workspace_elems,
              int accumulate, const FdAdamEpi* adams, int defer, int* splits_out, hipStream_t st) {
  if (splits_out) *splits_out = 0;
  long long slab_total = 0;
  bool fused = false;
  for (int i = 0; i < nprob; ++i) {
    slab_total += (long long)ps[i].M * ps[i].N;
    if (adams && adams[i].p) fused = true;
  }
  if (splits > 1 && workspace_elems < slab_total * splits) splits = 1;
  if (splits > 1 && fused) splits = 1;
  float* finals[2] = {(float*)ps[0].C, nprob > 1 ? (float*)ps[1].C : nullptr};
  long long off = 0;
  for (int i = 0; i < nprob; ++i) {
    GemmParams& p = ps[i];
    p.k_split = K / splits;
    p.accumulate = accumulate;
    if (adams) p.adam = adams[i];
    if (splits == 1) {
      p.out = finals[i]; p.slab_stride = 0;
    } else {
      p.C = workspace + off; p.slab_stride = (long long)p.M * p.N; p.ldc = p.N;
      off += p.slab_stride * splits;
      p.out = nullptr;
    }
  }
  if (!launch_id<false, false, EPI_F32>(ps[0], id, splits, st, nprob > 1 ? &ps[1] : nullptr)) return 7;
  if (splits > 1 && defer) {  // the caller reduces the slabs later (fd_splitk_reduce_batched)
    if (splits_out) *splits_out = splits;
    return 0;
  }
  if (splits > 1) {
    for (int i = 0; i < nprob; ++i) {
      const long long n4 = ps[i].slab_stride / 4;
      const int blocks = (int)std::min<long long>((n4 + 255) / 256, 2048);
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, (const float*)ps[i].C, finals[i], n4,
                         ps[i].slab_stride, splits, accumulate);
    }
  }
  return 0;
}

}  // namespace

// ---------------------------------------------------------------- C ABI
extern "C" {

// Copy the diagnostic stamps (FD_GEMM_STAMPS builds) of blocks [0, nblocks) to host memory
// [nblocks][8]; -1 in a normal build.
int fd_gemm_stamps(unsigned long long* host, int nblocks) {
#if FD_GEMM_STAMPS
  if (nblocks > STAMP_MAXB) nblocks = STAMP_MAXB;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 8 * nblocks, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? nblocks : -2;
#else
  (void)host; (void)nblocks;
  return -1;
#endif
}

// Force a configuration id / split count for a GEMM kind (tuning; -1 = auto).
int fd_gemm_set_cfg(int kind, int cfg, int splits) {
  if (kind < 0 || kind > 2 || cfg < -1 || cfg >= NCFG || (cfg >= 0 && !cfg_instantiated(cfg))) return 1;
  g_cfg_override[kind] = cfg;
  if (kind == 2) g_splits_override = splits;
  return 0;
}

// kind: 0 = NT (y = x W^T), 1 = NN (dx = dy W), 2 = TN (dW = dy^T x, fp32 out)
// Returns 0 on success, nonzero on unsupported shape.
int fd_gemm_ex(int kind, int epi, const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
               int ldc, const float* bias, void* aux, int ldaux, const void* res, int ldres, float* workspace,
               long long workspace_elems, int accumulate, const FdAdamEpi* adam,
               float* colsum, int* colsum_blocks, void* aux_out, hipStream_t st);

int fd_gemm(int kind, int epi, const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
            const float* bias, void* aux, int ldaux, const void* res, int ldres, float* workspace,
            long long workspace_elems, int accumulate, const FdAdamEpi* adam,
            float* colsum, int* colsum_blocks, hipStream_t st) {
  return fd_gemm_ex(kind, epi, A, B, C, M, N, K, lda, ldb, ldc, bias, aux, ldaux, res, ldres, workspace,
                    workspace_elems, accumulate, adam, colsum, colsum_blocks, nullptr, st);
}

// The next fd_gemm_ex launch on this host thread touches `pf` in its epilogue (GemmParams::ln.pf:
// staged_epilogue's pf_issue) -- the following launch's weight, so it comes from MALL / L2.
thread_local const char* g_gemm_pf = nullptr;
thread_local long long g_gemm_pf_bytes = 0;
int fd_gemm_pf(const void* pf, long long bytes) {
  g_gemm_pf = reinterpret_cast<const char*>(pf);
  g_gemm_pf_bytes = pf ? bytes : 0;
  return 0;
}

// fd_gemm + aux_out: the GELU' epilogue also re-creates gelu(aux) (nullable; EPI_GELU_BWD only).
int fd_gemm_ex(int kind, int epi, const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
               int ldc, const float* bias, void* aux, int ldaux, const void* res, int ldres, float* workspace,
               long long workspace_elems, int accumulate, const FdAdamEpi* adam,
               float* colsum, int* colsum_blocks, void* aux_out, hipStream_t st) {
  // the armed prefetch belongs to THIS call whatever happens below (never to a later launch)
  const char* pf = g_gemm_pf;
  const long long pf_bytes = g_gemm_pf_bytes;
  g_gemm_pf = nullptr;
  g_gemm_pf_bytes = 0;
  if (K % BKT != 0 || N % 64 != 0 || M <= 0 || kind < 0 || kind > 2 || epi >= EPI_LN) return 1;
  if (aux_out && (epi != EPI_GELU_BWD || kind == 2)) return 7;
  GemmParams p{};
  p.ln.pf = pf;
  p.ln.pf_bytes = pf_bytes;
  p.aux_out = (bf16_t*)aux_out;
  p.A = (const bf16_t*)A; p.B = (const bf16_t*)B; p.C = C;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.bias = bias; p.aux = (bf16_t*)aux; p.ldaux = ldaux; p.res = (const bf16_t*)res; p.ldres = ldres;
  p.k_split = K;
  {
    static const int diag = [] { const char* e = getenv("FD_GEMM_DIAG"); return e ? atoi(e) : 0; }();
    p.diag = diag;
  }
  int id = cfg_override(kind);
  if (id < 0) id = pick_cfg(kind, M, N, K);
  // Group height: A-panels of gm x BM rows x K (bf16) should take ~half of a 4 MiB L2.
  {
    const long long panel = (long long)CFGS[id].bm * K * 2;
    int gm = (int)std::max(1ll, std::min(16ll, (2ll << 20) / panel));
    const char* e = getenv("FD_GEMM_GROUP_M");
    if (e) gm = atoi(e);
    p.group_m = std::max(1, gm);
  }
  if (colsum) {
    // only the staged-fp32 epilogues sum columns: 128 x {128, 64} tiles (never 256-row ones)
    if (epi != EPI_GELU_BWD && epi != EPI_ADD) return 2;
    if (kind != 0 && kind != 1) return 2;
    // small-M 64-row tiles: 128 x 64; M >= 3584 (the 256-row pick): 128 x 128 -- the GELU' dX at M = 5184
    // 44.7 vs 49.3 us (128 x 64), profiles/r6_gemm_cfg_sweep_ffn_large_m.txt
    if (CFGS[id].bm != 128 && cfg_override(kind) < 0) id = (CFGS[id].bm > 128 && N % 128 == 0) ? 1 : 8;
    if (CFGS[id].bm != 128 || (CFGS[id].bn != 128 && CFGS[id].bn != 64) || N % CFGS[id].bn) {
      // the shape's tile has no staged-fp32 epilogue (e.g. 256 x 192 at M >= 3.5 k): launch
      // nothing, report 0 blocks -- the caller runs the plain GEMM + a column-sum pass
      if (colsum_blocks) *colsum_blocks = 0;
      return 0;
    }
    p.colsum = colsum;
    if (colsum_blocks) *colsum_blocks = (M + CFGS[id].bm - 1) / CFGS[id].bm;
  }
  // (NN launches fall back to cfg 8 below when the picked tile does not fit; that keeps 128 x 64)
  if (kind == 0) {  // K-major B: GELU' / residual epilogues as in the NN dX kind
    if (epi == EPI_F32) return 2;
    if (launch_epi<true, true>(epi, p, id, 1, st)) return 0;
    return launch_epi<true, true>(epi, p, 0, 1, st) ? 0 : 2;  // 128x64 fits any N % 64 == 0
  }
  if (kind == 1) {
    if (epi != EPI_BF16 && epi != EPI_GELU_BWD && epi != EPI_ADD) return 2;
    if (launch_epi<true, false>(epi, p, id, 1, st)) return 0;
    return launch_epi<true, false>(epi, p, 0, 1, st) ? 0 : 2;
  }
  // kind 2: dW[M=out][N=in] fp32.  Split K (the token dim) until the grid covers
  // the chip; slabs go to `workspace` and are reduced deterministically.
  if (M % 128 != 0) return 3;
  if (N % CFGS[id].bn != 0 || M % CFGS[id].bm != 0) id = 8;
  const long long tiles = tiles_of(id, M, N);
  int splits = 1;
  const int so = splits_override();
  if (so > 0) {
    splits = so;
    if (K % (splits * BKT) != 0) return 6;
  } else {
    while (tiles * splits < 400 && (K / (splits * 2)) % BKT == 0 && K / (splits * 2) >= 512) splits *= 2;
  }
  if (ldc != N) return 4;
  return dw_launch(&p, 1, id, splits, K, workspace, workspace_elems, accumulate, adam, 0, nullptr, st);
}

// QKV projection (x [M][K] W^T [N = 3 H 64][K] + bias -> qkv bf16) fused with the S <= 128 attention
// forward (fd_attn_fwd's arguments) in ONE launch (gemm_attn_fwd_kernel).  flags: >= tiles granules
// (int64, zeroed once), cnt the LayerNorm exchange epoch, err its timeout flag, xsite < FD_LN_XSITES - 1
// unique per launch within an epoch.  Nothing is launched on a non-zero return.
int fd_gemm_attn_fwd(const void* x, const void* w, const float* bias, void* qkv, int M, int K, const float* kbias,
                     void* ctx, float* lse, int B, int S, int H, const uint32_t* seed_ptr, uint32_t site, uint32_t thr,
                     float drop_scale, const int* cu, int rows, uint64_t* dmask, int q_live, void* cxc, void* xc,
                     const void* xres, int Bp, uint64_t* flags, int nflags, const int* cnt, int xsite, int* err,
                     int mode, int split, hipStream_t st) {
  const char* pf = g_gemm_pf;  // (an armed prefetch belongs to this call whatever happens below)
  const long long pf_bytes = g_gemm_pf_bytes;
  g_gemm_pf = nullptr;
  g_gemm_pf_bytes = 0;
  const int D = H * DH, N = 3 * D;
  if (mode != 1 && mode != 2) return 6;
  // split 2 (S > 128, varlen): the caller knows every sequence has <= 128 tokens (attention.hip split_mode)
  const bool sh = split == 2 && cu && S <= 512 && mode == 2;
  if (M <= 0 || K % BKT || N % QA_BN || S % 64 || (S > 128 && !sh) || B <= 0 || !bias || !flags || !cnt || !err)
    return 1;
  if (xsite < 0 || xsite >= FD_LN_XSITES - 1) return 2;
  if ((cu ? rows : B * S) != M || (long long)M * N * 2 >= (1ll << 31)) return 3;
  if (cxc && (!xc || !xres || q_live != 1 || Bp < B)) return 4;
  const int tiles_n = N / QA_BN, ntiles = ((M + QA_BM - 1) / QA_BM) * tiles_n;
  if (ntiles > nflags) return 5;
  GemmParams p{};
  p.ln.pf = pf;
  p.ln.pf_bytes = pf_bytes;
  p.A = (const bf16_t*)x; p.B = (const bf16_t*)w; p.C = qkv;
  p.M = M; p.N = N; p.K = K; p.lda = K; p.ldb = K; p.ldc = N;
  p.bias = bias;
  p.k_split = K;
  p.group_m = (int)std::max(1ll, std::min(16ll, (2ll << 20) / ((long long)QA_BM * K * 2)));  // (as fd_gemm_ex)
  AttnArgs a{};
  a.cxc = (bf16_t*)cxc; a.xc = (bf16_t*)xc; a.xres = (const bf16_t*)xres; a.Bp = Bp;
  a.q_live = q_live;
  a.cu = cu;
  a.dmask = dmask;
  a.qkv = (const bf16_t*)qkv; a.kbias = kbias; a.ctx = (bf16_t*)ctx; a.lse = lse;
  a.seed_ptr = seed_ptr; a.site = site; a.drop_threshold = thr; a.drop_scale = drop_scale;
  a.B = B; a.S = S; a.H = H; a.scale = 0.125f; a.rows = rows;
  a.split = S > 128 ? 1 : 0;  // (a sequence past 128 tokens is skipped, never staged past the LDS images)
  const int items = H * (B + (cu ? 1 : 0));
  if (mode == 2) {  // per-(sequence, head) projection + attention (no hand-off, no flags)
    // (sequence-major: an XCD's blocks share their sequences' x rows in its L2 -- -5 us per step over
    //  4 pairs against head-major, profiles/r6_ab_fused_qkv_attention.txt)
    static const int seq_major = [] { const char* e = getenv("FD_SEQATTN_SEQ_MAJOR"); return e ? atoi(e) : 1; }();
    SeqQkvArgs g{(const bf16_t*)x, (const bf16_t*)w, bias, M, K, seq_major};
    hipLaunchKernelGGL(seq_attn_fwd_kernel, dim3(items), dim3(512), 0, st, g, a);
    return 0;
  }
  QkvAttnSync q{flags, cnt, err, xsite, ntiles, tiles_n};
  hipLaunchKernelGGL(gemm_attn_fwd_kernel, dim3(ntiles + items), dim3(64 * QA_NW), 0, st, p, a, q);
  return 0;
}

// The S <= 128 attention backward with the out-projection's dX computed per (sequence, head) inside
// it (attn_bwd_proj_kernel): fd_attn_bwd's arguments with dctx replaced by dy [M][K] and the
// out-projection weight W [K][D].  splits: the K splits of the GEMM it stands in for (1: one chain;
// the pruned block's M <= 64 split-K slabs otherwise, summed in split order -- bitwise either way).
// dresc / dres (the pruned block's compact [CLS] form, q_live 1): dy holds the [CLS] rows.
int fd_attn_bwd_proj(const void* qkv, const float* kbias, const void* ctx, const float* lse, const void* dy,
                     const void* w, int M, int K, int splits, void* dqkv, int B, int S, int H,
                     const uint32_t* seed_ptr, uint32_t site, uint32_t thr, float drop_scale, const int* cu, int rows,
                     const uint64_t* dmask, const void* dresc, void* dres, int split, hipStream_t st) {
  const bool sh = split == 2 && cu && S <= 512;  // (as fd_gemm_attn_fwd)
  if (S % 64 || (S > 128 && !sh) || K % BKT || M <= 0 || B <= 0 || !dy || !w || splits <= 0 || (K / BKT) % splits) return 1;
  // compact [CLS] form: dy = the [CLS] rows' out-projection gradient [M >= B][K]; q_live 1
  if ((dresc != nullptr) != (dres != nullptr) || (dres ? M < B : (cu ? rows : B * S) != M)) return 2;
  AttnArgs a{};
  a.dresc = (const bf16_t*)dresc; a.dres = (bf16_t*)dres;
  a.q_live = dres ? 1 : 0;
  a.cu = cu;
  a.dmask = const_cast<uint64_t*>(dmask);
  a.qkv = (const bf16_t*)qkv; a.kbias = kbias; a.ctx = (bf16_t*)ctx; a.lse = (float*)lse;
  a.dqkv = (bf16_t*)dqkv;
  a.seed_ptr = seed_ptr; a.site = site; a.drop_threshold = thr; a.drop_scale = drop_scale;
  a.B = B; a.S = S; a.H = H; a.scale = 0.125f; a.rows = rows;
  a.split = S > 128 ? 1 : 0;
  static const int order = [] { const char* e = getenv("FD_ATTNBWD_SEQ_MAJOR"); return e ? atoi(e) : 1; }();
  OProjArgs pj{(const bf16_t*)dy, (const bf16_t*)w, M, K, K / BKT / splits, order};
  hipLaunchKernelGGL(attn_bwd_proj_kernel, dim3(H * (B + (cu ? 1 : 0))), dim3(512), 0, st, a, pj);
  return 0;
}

// Split-K NT product into fp32 slabs: slabs[z][M][N] = A[M][k in split z] Bt[N][k in split z]^T
// (A [M][lda], Bt [N][ldb] bf16, K % (64 * splits) == 0), one launch of splits x tiles blocks --
// the small-M GEMMs (the pruned block's [CLS] rows) on the whole chip instead of a dozen CUs.
// The caller reduces the slabs and applies the epilogue (splitk.hip fd_splitk_epilogue).
// splits <= 0: picked here (largest divisor of K / 64 that keeps >= 2 K tiles per block and the
// grid within one round of 256 blocks); returns the split count used, or a negative error.
int fd_gemm_f32_splits(const void* A, const void* Bt, float* slabs, long long slab_elems, int M, int N, int K,
                       int lda, int ldb, int splits, int b_mn, hipStream_t st) {
  // b_mn: Bt is the weight W [K][N] itself (MN-major B, ldb = its row pitch)
  if (M <= 0 || K % BKT || N % 64 || !A || !Bt || !slabs) return -1;
  const int id = M <= 64 ? 13 : 8;
  const long long tiles = tiles_of(id, M, N);
  const int nkt = K / BKT;
  if (splits <= 0) {
    splits = 1;
    for (int s = 1; s <= nkt; ++s)
      if (nkt % s == 0 && tiles * s <= 256 && nkt / s >= 2) splits = s;
  }
  if (nkt % splits || slab_elems < (long long)splits * M * N) return -2;
  GemmParams p{};
  p.A = (const bf16_t*)A; p.B = (const bf16_t*)Bt; p.C = slabs;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = N;
  p.k_split = K / splits;
  p.slab_stride = (long long)M * N;
  p.group_m = 1;
  if (b_mn) return launch_id<true, false, EPI_F32>(p, id, splits, st) ? splits : -3;
  return launch_id<true, true, EPI_F32>(p, id, splits, st) ? splits : -3;
}

// Two weight-gradient GEMMs over the same token dimension in ONE launch:
//   C0[M0][N0] (+)= A0^T B0,  C1[M1][N1] (+)= A1^T B1   (A_i [K][M_i], B_i [K][N_i] bf16; C_i fp32)
// Split K only while the combined grid is under one round; slabs of problem 0 then 1.
// K splits fd_gemm_dw2 plans for these shapes (<= 0: unsupported) -- lets the caller size a
// slab buffer of its own for a deferred reduce.
// Tile configuration of a grouped dW pair.  Default 128 x 64 (cfg 8); pairs too small to give
// 400 such tiles (o + qkv: 288) use FD_GEMM_DW_SMALL_CFG, the others FD_GEMM_DW_BIG_CFG
// (-1 = cfg 8).  A 64 x 64 small-pair grid has 576 tiles, so it runs unsplit: no fp32 slabs,
// no reduce (scripts/dw_split_probe.py).
int dw2_cfg(int M0, int N0, int M1, int N1) {
  int id = cfg_override(2);
  if (id < 0) {
    static const int small_cfg = [] { const char* e = getenv("FD_GEMM_DW_SMALL_CFG"); return e ? atoi(e) : -1; }();
    static const int big_cfg = [] { const char* e = getenv("FD_GEMM_DW_BIG_CFG"); return e ? atoi(e) : -1; }();
    const bool small = tiles_of(8, M0, N0) + tiles_of(8, M1, N1) < 400;
    id = small ? small_cfg : big_cfg;
    if (!cfg_instantiated(id)) id = 8;
  }
  if (M0 % CFGS[id].bm || M1 % CFGS[id].bm || N0 % CFGS[id].bn || N1 % CFGS[id].bn) id = 8;
  return id;
}

int fd_gemm_dw2_splits(int M0, int N0, int M1, int N1, int K) {
  const int id = dw2_cfg(M0, N0, M1, N1);
  const long long tiles = tiles_of(id, M0, N0) + tiles_of(id, M1, N1);
  int splits = 1;
  const int so = splits_override();
  if (so > 0) {
    splits = so;
    if (K % (splits * BKT) != 0) return 0;
  } else {
    while (tiles * splits < 400 && (K / (splits * 2)) % BKT == 0 && K / (splits * 2) >= 512) splits *= 2;
  }
  return splits;
}

int fd_gemm_dw2(const void* A0, const void* B0, float* C0, int M0, int N0, const void* A1, const void* B1, float* C1,
                int M1, int N1, int K, float* workspace, long long workspace_elems, int accumulate,
                const FdAdamEpi* adams, int defer, int* splits_out, hipStream_t st) {
  if (K % BKT != 0 || M0 % 128 || M1 % 128 || N0 % 64 || N1 % 64 || M0 <= 0 || M1 <= 0) return 1;
  const int id = dw2_cfg(M0, N0, M1, N1);
  static const int diag = [] { const char* e = getenv("FD_GEMM_DIAG"); return e ? atoi(e) : 0; }();
  GemmParams p[2]{};
  const void* As[2] = {A0, A1};
  const void* Bs[2] = {B0, B1};
  float* Cs[2] = {C0, C1};
  const int Ms[2] = {M0, M1}, Ns[2] = {N0, N1};
  const long long panel = (long long)CFGS[id].bm * K * 2;
  const int gm = (int)std::max(1ll, std::min(16ll, (2ll << 20) / panel));
  for (int i = 0; i < 2; ++i) {
    p[i].A = (const bf16_t*)As[i]; p[i].B = (const bf16_t*)Bs[i]; p[i].C = Cs[i];
    p[i].M = Ms[i]; p[i].N = Ns[i]; p[i].K = K; p[i].lda = Ms[i]; p[i].ldb = Ns[i]; p[i].ldc = Ns[i];
    p[i].group_m = gm; p[i].diag = diag;
  }
  const int splits = fd_gemm_dw2_splits(M0, N0, M1, N1, K);
  if (splits <= 0) return 6;
  return dw_launch(p, 2, id, splits, K, workspace, workspace_elems, accumulate, adams, defer, splits_out, st);
}

// All-layer weight gradients in one launch (gemm_dw_batch_kernel).  probs[i] = {A, B, C, p, m,
// v, sh, M, N, -, accumulate} (tile0 is filled here); adam != nullptr -> hyper-parameters of
// the fused optimizer step for the problems with p != nullptr.  cfg < 0: FD_GEMM_DWB_CFG or
// the default 256 x 256 (2 x 4 waves, 2-deep ring, banded fp32 epilogue; falls back to 128 x 64
// when a shape is not a multiple of 256).  Measured (profiles/r2_dw_batch_isolated_cfgs.txt,
// all 24 dW of the bs32 step + Adam): 256^2 448 us, 128^2 470 us, 128 x 64 492 us.  Returns 0, or nonzero on an unsupported
// shape (nothing launched).
bool dwb_launch_cfg(int id, DwBatch& bt, hipStream_t st, bool dry) {
  auto go = [&](auto kern, int bm, int bn, int threads) {
    for (int i = 0; i < bt.n; ++i)
      if (bt.pr[i].M % bm || bt.pr[i].N % (bt.pr[i].half ? DWB_HBN : bn)) return false;
    int t = 0;
    for (int i = 0; i < bt.n; ++i) {
      bt.pr[i].tile0 = t;
      t += (bt.pr[i].M / bm) * (bt.pr[i].N / (bt.pr[i].half ? DWB_HBN : bn));
    }
    bt.ntiles = t;
    const int nblk = bt.mixed ? 8 * (bt.cls_pad[0] + bt.cls_pad[1] + bt.cls_pad[2]) : t;
    if (!dry) hipLaunchKernelGGL(kern, dim3(nblk + bt.rest.flat_blocks + bt.rest.row_blocks), dim3(threads), 0, st, bt);
    return true;
  };
  if (bt.mixed && id != 11) return false;
  switch (id) {
    case 1: return go(gemm_dw_batch_kernel<128, 128, 2, 2, 2>, 128, 128, 256);
    case 8: return go(gemm_dw_batch_kernel<128, 64, 2, 2, 2>, 128, 64, 256);
    case 11: return go(gemm_dw_batch_kernel<256, 256, 2, 4, 2, BKT, true>, 256, 256, 512);
  }
  return false;
}

// FD_DWB_MIX / fd_gemm_dwb_set_mix: 0 off, 1 (default) when it shortens the schedule, 2 forced
// (tests: any launch with at least two long problems gets a half-tile class)
int g_dwb_mix = -1;
long long g_dwb_mixed_launches = 0;  // (tests: proof the mixed schedule ran)

int dwb_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess)
      n = 0;
    return n > 0 ? n : 256;
  }();
  return cus;
}

// The all-layer launch's tile rounds (256 x 256 tiles, one block per CU).  The bs32 step has 567
// long tiles (K = the packed tokens) and 81 short ones (the pruned block's K = 64 [CLS] rows): with
// the XCD remap's equal-count ranges XCD 0 got every short tile and XCDs 1..7 81 long tiles each --
// three rounds of long tiles, the third at 17 / 32 occupancy.  Plan instead: long tiles in whole
// rounds, the excess long work E as 256 x 128 half tiles of whole problems (the smallest subset of
// long problems holding >= E tiles), and every class dealt evenly over the XCDs, so the half and
// short tiles share ONE partial round.  Returns whether it applies (else the launch is unchanged).
bool plan_dwb_mix(DwBatch& bt, int mode) {
  if (mode <= 0 || bt.n < 2) return false;
  const int cus = dwb_cus();
  int kmax = 0;
  for (int i = 0; i < bt.n; ++i) kmax = std::max(kmax, bt.pr[i].K > 0 ? bt.pr[i].K : bt.K);
  int cls[DWB_MAXP], tiles[DWB_MAXP], L = 0, Sh = 0, nlong = 0;
  for (int i = 0; i < bt.n; ++i) {
    const DwProb& q = bt.pr[i];
    if (q.M % 256 || q.N % 256) return false;
    const int k = q.K > 0 ? q.K : bt.K;
    tiles[i] = (q.M / 256) * (q.N / 256);
    cls[i] = 8 * k <= kmax ? 2 : 0;
    if (cls[i] == 0) { L += tiles[i]; ++nlong; } else Sh += tiles[i];
  }
  if (nlong < 2) return false;
  const int rounds = L / cus, E = L - rounds * cus;
  int target = E;
  if (mode == 1 && (rounds == 0 || E == 0)) return false;
  if (mode == 2) target = 1;  // forced (tests): the smallest long problem goes to half tiles
  // smallest subset sum >= target over the long problems (reachable sums; <= 32 problems)
  std::vector<int> from(L + 1, -2);  // from[s]: last problem added to reach sum s (-1: empty set)
  from[0] = -1;
  std::vector<int> used_at(L + 1, 0);
  for (int i = 0; i < bt.n; ++i) {
    if (cls[i]) continue;
    for (int s = L; s >= tiles[i]; --s)
      if (from[s] == -2 && from[s - tiles[i]] != -2 && s - tiles[i] >= 0) {
        // (0/1 knapsack, descending s: problem i is used at most once per reachable sum)
        from[s] = i;
        used_at[s] = s - tiles[i];
      }
  }
  int best = -1;
  for (int s = target; s <= L; ++s)
    if (from[s] != -2 && s < L) { best = s; break; }
  if (best < 0) return false;
  // the half + short tiles must fit the partial round's free blocks per XCD
  const int per = cus / 8;
  const int big_x = (L - best + 7) / 8, tail_x = (2 * best + 7) / 8 + (Sh + 7) / 8;
  const int free_x = (rounds * per > big_x ? rounds * per - big_x : 0) + per;
  if (mode == 1 && (big_x > rounds * per || tail_x > free_x)) return false;
  for (int s = best; s > 0; s = used_at[s]) cls[from[s]] = 1;
  // stable reorder by class, in dispatch order: long full tiles, long half tiles, short -- or, with
  // FD_DWB_SHORT_FIRST=1 (A/B), the short tiles (a one-step K loop + a full Adam epilogue: HBM-bound)
  // first, beside the first round's operand-bound K loops
  static const int short_first = [] { const char* e = getenv("FD_DWB_SHORT_FIRST"); return e ? atoi(e) : 1; }();
  int order[3] = {short_first ? 2 : 0, short_first ? 0 : 1, short_first ? 1 : 2};
  // FD_DWB_CLASS_ORDER=<3 digits> (A/B): any dispatch order of the classes 0 long, 1 half, 2 short
  static const char* class_order = getenv("FD_DWB_CLASS_ORDER");
  if (class_order && strlen(class_order) == 3) {
    int o[3], seen = 0;
    for (int q = 0; q < 3; ++q) {
      o[q] = class_order[q] - '0';
      if (o[q] >= 0 && o[q] < 3) seen |= 1 << o[q];
    }
    if (seen == 7)
      for (int q = 0; q < 3; ++q) order[q] = o[q];
  }
  DwProb pr[DWB_MAXP];
  int k = 0, off = 0;
  for (int q = 0; q < 3; ++q) {
    const int c = order[q];
    int t = 0;
    for (int i = 0; i < bt.n; ++i)
      if (cls[i] == c) {
        pr[k] = bt.pr[i];
        pr[k].half = c == 1;
        ++k;
        t += c == 1 ? 2 * tiles[i] : tiles[i];
      }
    bt.cls_tiles[q] = t;
    bt.cls_pad[q] = (t + 7) / 8;
    bt.cls_off[q] = off;
    off += t;
  }
  for (int i = 0; i < bt.n; ++i) bt.pr[i] = pr[i];
  bt.mixed = 1;
  return true;
}

int fd_gemm_dw_batch(int n, const DwProb* probs, int K, const int* step, const float* hyper, int cfg,
                     const FdAdamRest* rest, hipStream_t st) {
  if (n <= 0 || n > DWB_MAXP || K <= 0 || K % BKT) return 1;
  DwBatch bt{};
  if (rest && rest->p) {
    if (!hyper || !step || !rest->g || !rest->m || !rest->v || (rest->nruns > 0) != (rest->runs != nullptr) ||
        rest->n4 < 0 || (rest->ever && (rest->wrows <= 0 || rest->wrow4 <= 0 || rest->woff % 4)))
      return 7;
    bt.rest = *rest;
    // ~4 float4 per thread of the run table; one 64-row flag chunk per wave of the word table
    bt.rest.flat_blocks = rest->n4 > 0 ? (int)std::min<long long>(128, (rest->n4 + 2047) / 2048) : 0;
    bt.rest.row_blocks = rest->ever ? std::min(128, (rest->wrows + 127) / 128) : 0;
    // (FD_DW_REST_FIRST=0: after the tiles; leading measured 1.6395 / 1.6434 vs 1.6452 / 1.6436 ms/step,
    // profiles/r5_ab_adam_in_dw.txt)
    static const int first = [] { const char* e = getenv("FD_DW_REST_FIRST"); return e ? atoi(e) : 1; }();
    bt.rest.first = first;
    if (first) {  // (a multiple of 8 blocks in all)
      const int pad = (8 - (bt.rest.flat_blocks + bt.rest.row_blocks) % 8) % 8;
      bt.rest.row_blocks += pad;
    }
  }
  bt.n = n;
  bt.K = K;
  static const int diag = [] { const char* e = getenv("FD_GEMM_DIAG"); return e ? atoi(e) : 0; }();
  bt.diag = diag;
  for (int i = 0; i < n; ++i) {
    bt.pr[i] = probs[i];
    if (!probs[i].A || !probs[i].B || (!probs[i].C && !probs[i].p) || probs[i].M <= 0 || probs[i].N <= 0) return 2;
    if (probs[i].K < 0 || probs[i].K % BKT) return 5;
    if (probs[i].p && (!probs[i].m || !probs[i].v || !step || !hyper)) return 3;
  }
  if (hyper) {
    bt.step = step;
    bt.lr = hyper[0]; bt.b1 = hyper[1]; bt.b2 = hyper[2]; bt.eps = hyper[3]; bt.wd = hyper[4];
    bt.decoupled = hyper[5] != 0.f;
  }
  int id = cfg;
  if (id < 0) {
    static const int env = [] { const char* e = getenv("FD_GEMM_DWB_CFG"); return e ? atoi(e) : -1; }();
    id = env >= 0 ? env : 11;
  }
  // Group height: every tile row of a problem (column-major tile order, so consecutive tiles -- one
  // XCD after the remap -- share the B panel of a column).  In the step 1.585 vs 1.605 ms/step
  // against the earlier ~half-an-L2 heuristic (3 rows at K = 2688); 12, 16, 24 and 64 alike
  // (profiles/r5_ab_dwb_group_m.txt; isolated, with operands not just written by the backward, no
  // difference).
  bt.group_m = 64;
  static const int gm_env = [] { const char* e = getenv("FD_DWB_GROUP_M"); return e ? atoi(e) : 0; }();
  if (gm_env > 0) bt.group_m = gm_env;  // tuning override
  if (g_dwb_mix < 0) {
    const char* e = getenv("FD_DWB_MIX");
    g_dwb_mix = e ? atoi(e) : 1;
  }
  if (id == 11 && plan_dwb_mix(bt, g_dwb_mix) && !dwb_launch_cfg(id, bt, st, true)) {
    // (a shape the half tiles do not cover: the plain schedule)
    bt.mixed = 0;
    for (int i = 0; i < n; ++i) bt.pr[i] = probs[i];
  }
  if (bt.mixed) ++g_dwb_mixed_launches;
  if (!dwb_launch_cfg(id, bt, st, true)) {
    id = 8;  // 128 x 64 fits every supported shape (M % 128, N % 64)
    if (!dwb_launch_cfg(id, bt, st, true)) return 4;
  }
  dwb_launch_cfg(id, bt, st, false);
  return 0;
}

// Reduce n deferred split-K weight gradients (slab layout of fd_gemm_dw2) in one launch.
int fd_splitk_reduce_batched(int n, const float* const* slabs, float* const* outs, const long long* numel,
                             const int* splits, const int* accumulate, hipStream_t st) {
  for (int base = 0; base < n; base += RED_MAXJ) {
    ReduceBatch rb{};
    rb.n = std::min(RED_MAXJ, n - base);
    int blocks = 0;
    for (int i = 0; i < rb.n; ++i) {
      const int k = base + i;
      if (numel[k] % 4 || splits[k] < 1) return 1;
      rb.j[i] = ReduceJob{slabs[k], outs[k], numel[k] / 4, numel[k], splits[k], accumulate[k]};
      rb.start[i] = blocks;
      blocks += (int)std::min<long long>((numel[k] / 4 + 1023) / 1024, 1024);  // ~4 float4 per thread
    }
    rb.start[rb.n] = blocks;
    hipLaunchKernelGGL(splitk_reduce_batched_kernel, dim3(blocks), dim3(256), 0, st, rb);
  }
  return 0;
}


// LayerNorm-fused NT GEMM: C[M][N] = epilogue(A[M][K] Bt[N][K]^T) with N = the hidden size
// (FdLnEpi, adam_epi.h).  bwd = 0: EPI_LN (bias + dropout + residual + LN), 1: EPI_LN_BWD.
// cfg < 0: FD_GEMM_LN_CFG or 24 (128 x 64, 8 waves, two K tiles per barrier -- the N = 768
// configuration of the plain GEMM).  Returns the number of row blocks (the colpart rows),
// or a negative code on an unsupported shape (nothing launched).
long long fd_gemm_dwb_mixed_launches() { return g_dwb_mixed_launches; }

int fd_gemm_dwb_set_mix(int mode) {
  const int old = g_dwb_mix;
  g_dwb_mix = mode;
  return old;
}

int fd_gemm_ln_set_diag(int diag) {
  g_ln_diag = diag;
  return 0;
}

int fd_gemm_ln(int bwd, const void* A, const void* Bt, void* C, int M, int N, int K, const float* bias,
               const void* res, int ldres, const FdLnEpi* ln, int cfg, int b_mn, hipStream_t st) {
  if (M <= 0 || K % BKT || N % 64 || !ln || !res || (!bwd && !bias)) return -1;
  // b_mn: B is the weight W [K][N] itself (MN-major; LayerNorm backward only)
  if (b_mn && !bwd) return -6;
  if (ln->xsite >= FD_LN_XSITES) return -5;
  int id = cfg;
  if (id < 0) {
    static const int env = [] { const char* e = getenv("FD_GEMM_LN_CFG"); return e ? atoi(e) : -1; }();
    id = env >= 0 ? env : (M <= 64 && smallm_tiles() ? 13 : 24);
  }
  // two-K-half tiles (gemm_ln2_kernel): FD_GEMM_LN2_MINK (default 2048) <= K, needs the exchange
  // buffers; the grid stays one resident round (2 blocks per 128 x 128 tile = one per 128 x 64)
  static const int ln2_mink = [] { const char* e = getenv("FD_GEMM_LN2_MINK"); return e ? atoi(e) : 2048; }();
  const bool ln2_ok = cfg < 0 && id == 24 && K % 128 == 0 && N % 128 == 0 && ln->xbuf && ln->xflag;
  bool ln2 = ln2_ok && ln2_mink > 0 && K >= ln2_mink;
  int bm = id == 13 ? 64 : 128;
  const int bn = 64;
  if (N / bn > LN_MAXK * (bn / 8)) return -2;
  {
    // one resident round: no more tiles than CUs (cfg 24: one 147 KiB block per CU)
    static const int cus = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                   hipSuccess)
        n = 0;
      return n;
    }();
    const int max_tiles = std::min(LN_MAX_TILES, cus > 0 ? cus : LN_MAX_TILES);
    if (((M + bm - 1) / bm) * (N / bn) > max_tiles) {
      // too many 128-row tiles for one round: 256-row two-K-half tiles (any K), else the caller
      // takes the unfused kernels
      if (!ln2_ok || ((M + 255) / 256) * (N / bn) > max_tiles) return -4;
      bm = 256;
      ln2 = true;
    }
  }
  GemmParams p{};
  p.A = (const bf16_t*)A; p.B = (const bf16_t*)Bt; p.C = C;
  p.M = M; p.N = N; p.K = K; p.lda = K; p.ldb = b_mn ? N : K; p.ldc = N;
  p.bias = bias; p.res = (const bf16_t*)res; p.ldres = ldres;
  p.k_split = K;
  p.ln = *ln;
  if (g_ln_diag < 0) {
    const char* e = getenv("FD_GEMM_LN_DIAG");
    g_ln_diag = e ? atoi(e) : 0;
  }
  // profiling / tests only: 16 = no row-block rendezvous (wrong statistics), 64 = force the
  // rendezvous timeout (fd_gemm_ln_set_diag; tests/test_fused_ln_gpu.py)
  p.diag = g_ln_diag;
  const int tiles_m = (M + bm - 1) / bm;
  const dim3 grid(tiles_m * (N / bn));
  auto go = [&](auto kern, int threads) { hipLaunchKernelGGL(kern, grid, dim3(threads), 0, st, p); };
  if (ln2) {  // (same grid: 2 blocks per 128 x 128 product tile = one per 128 x 64 LayerNorm tile)
    // (4 ring slots of 32 KiB; the whole 160 KiB as 5 slots measured slower: 1.630 vs 1.623 ms,
    //  profiles/r5_rejected_ab.txt)
    if (bm == 256) {
      if (b_mn) go(gemm_ln2_kernel<EPI_LN2_BWD, false, 256>, 512);
      else if (bwd) go(gemm_ln2_kernel<EPI_LN2_BWD, true, 256>, 512);
      else go(gemm_ln2_kernel<EPI_LN2, true, 256>, 512);
    } else {
      if (b_mn) go(gemm_ln2_kernel<EPI_LN2_BWD, false>, 512);
      else if (bwd) go(gemm_ln2_kernel<EPI_LN2_BWD, true>, 512);
      else go(gemm_ln2_kernel<EPI_LN2, true>, 512);
    }
    return tiles_m;
  }
#define FD_LN_CASE(ID, BM_, BN_, WM_, WN_, S_)                                          \
  case ID:                                                                             \
    if (b_mn) go(gemm_ln_kernel<BM_, BN_, EPI_LN_BWD, WM_, WN_, S_, false>, 64 * WM_ * WN_); \
    else if (bwd) go(gemm_ln_kernel<BM_, BN_, EPI_LN_BWD, WM_, WN_, S_>, 64 * WM_ * WN_);   \
    else go(gemm_ln_kernel<BM_, BN_, EPI_LN, WM_, WN_, S_>, 64 * WM_ * WN_);           \
    break;
  switch (id) {
    FD_LN_CASE(24, 128, 64, 4, 2, 6)
    FD_LN_CASE(0, 128, 64, 2, 2, 3)
    FD_LN_CASE(18, 128, 64, 4, 2, 3)
    FD_LN_CASE(13, 64, 64, 2, 2, 3)
    default: return -3;
  }
#undef FD_LN_CASE
  return tiles_m;
}

}  // extern "C"
