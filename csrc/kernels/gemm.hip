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
// Design (MI355X-first, cdna_hip_programming.md §5):
//  * 256 threads = 4 waves in a 2x2 grid; each wave owns a (BM/2)x(BN/2) tile of
//    16x16 MFMA sub-tiles; K tile 64 (two 32-deep MFMA steps).
//  * Operand tiles go HBM/L2 -> LDS with global_load_lds_dwordx4 (LDS-DMA, no
//    VGPR round trip, no ds_write issue cost), double-buffered: tile k+1's DMA
//    is issued before tile k's MFMAs; one vmcnt(0)+barrier per K tile.
//  * The DMA writes LDS lane-linearly, so bank-conflict swizzles are applied on
//    the per-lane SOURCE address and undone on the read (rule 21):
//    K-major images [rows][64] use chunk ^= (row>>1)&7 (conflict-free
//    ds_read_b128 fragments); MN-major images [64 k][BMN] are read with the
//    transposing ds_read_b64_tr_b16 (T10) and use chunk ^= fk(k) so the 16-lane
//    groups of each half-wave hit disjoint banks.
//  * Operands are swapped inside the MFMA (D = B^T A^T = C^T) so every lane owns
//    4 consecutive output columns: 8-byte bf16 / 16-byte fp32 stores, vectorised
//    bias / residual / GELU-aux loads in the epilogue.
//  * Host picks the tile (128x128 / 128x96 / 128x64) that best fills 256 CUs x
//    2 resident blocks; XCD-aware bijective block remap (T1).
#include "common.h"

#include <cstdlib>

namespace {

enum Epi : int {
  EPI_BF16 = 0,       // C(bf16) = acc
  EPI_BIAS = 1,       // C(bf16) = acc + bias[n]
  EPI_BIAS_GELU = 2,  // aux(bf16) = acc + bias[n];  C(bf16) = gelu(aux)
  EPI_GELU_BWD = 3,   // C(bf16) = acc * gelu'(aux[m][n])
  EPI_ADD = 4,        // C(bf16) = acc + res[m][n]
  EPI_F32 = 5,        // C(fp32 slab z) = acc
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
  int diag;              // FD_GEMM_DIAG bits (profiling only): 1 no in-loop DMA, 2 no MFMA, 4 no stores
};

// Logical tile id -> (tm, tn).  After the XCD remap each XCD owns a contiguous
// range of logical ids; walking them in groups of `gm` M-tiles x all N-tiles
// means the blocks resident on one XCD share gm A-panels and a few B-panels,
// a working set sized by the host to fit the XCD's 4 MiB L2 (instead of every
// XCD streaming all of A from the Infinity Cache).
DEV void tile_coords(int lid, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  const int per_group = gm * tiles_n;
  const int group = lid / per_group;
  const int first_m = group * gm;
  const int rows = min(gm, tiles_m - first_m);
  const int in_group = lid - group * per_group;
  tm = first_m + in_group % rows;
  tn = in_group / rows;
}

constexpr int BKT = 64;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

// Swizzle of 16-byte chunks for the MN-major ([k][mn]) LDS image.
template <int BMN>
DEV int fk(int k) {
  if constexpr (BMN == 128) return ((k & 3) | ((k >> 1) & 4)) << 1;
  else return (((k >> 1) & 1) | ((k >> 2) & 2)) << 1;
}

// K-major chunk swizzle: 128-byte rows (BK=64) -> chunk ^ ((r>>1)&7);
// 64-byte rows (BK=32) -> chunk ^ ((r>>2)&3).  Either way 16 consecutive rows
// reading the same logical chunk land on 16 distinct 16-byte bank slots.
template <int BK>
DEV int ksw(int r) {
  if constexpr (BK == 64) return (r >> 1) & 7;
  else return (r >> 2) & 3;
}

template <int ROWS, bool KMAJ, int BK = BKT, int NWAVES = 4>
struct Operand {
  static constexpr int BYTES = ROWS * BK * 2;              // one LDS buffer
  static constexpr int PER_WAVE = BYTES / 1024 / NWAVES;  // 1 KiB DMA pieces per wave per tile
  static constexpr int CH = KMAJ ? BK / 8 : ROWS / 8; // 16-byte chunks per LDS row
  static constexpr int ROWB = CH * 16;
  static_assert(KMAJ || ROWS == 64 || ROWS == 128, "MN-major tiles must be 64 or 128 wide");
  static_assert(PER_WAVE * NWAVES * 1024 == BYTES, "tile must split into whole 1 KiB pieces per wave");

  // LDS-DMA of the K tile starting at k0.  K-major rows beyond `lim` are clamped
  // (their products land in output rows that are never stored).
  DEV static void stage(const bf16_t* base, int ld, int row0, int k0, int lim, char* lds, int wid, int lane) {
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int piece = wid * PER_WAVE + i;
      const int pos = piece * 64 + lane;  // physical 16-byte chunk of the image
      const bf16_t* src;
      if constexpr (KMAJ) {
        const int r = pos / CH, c = (pos % CH) ^ ksw<BK>(r);
        const int gr = min(row0 + r, lim - 1);
        src = base + (size_t)gr * ld + k0 + c * 8;
      } else {
        const int k = pos / CH, c = (pos % CH) ^ fk<ROWS>(k);
        src = base + (size_t)(k0 + k) * ld + row0 + c * 8;
      }
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(lds + piece * 1024), 16, 0, 0);
    }
  }

  // MFMA fragment for rows [row0, row0+16) and k-step s (32 deep).
  DEV static bf16x8 frag(const char* lds, int row0, int s, int lane) {
    if constexpr (KMAJ) {
      const int row = row0 + (lane & 15);
      const int c = s * 4 + (lane >> 4);
      return *reinterpret_cast<const bf16x8*>(lds + row * ROWB + ((c ^ ksw<BK>(row)) << 4));
    } else {
      const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
      const int c = (row0 >> 3) + (p >> 1);
      bf16x8 out;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = s * 32 + 8 * g + 4 * h + q;
        const char* addr = lds + k * ROWB + ((c ^ fk<ROWS>(k)) << 4) + (p & 1) * 8;
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

template <int EPI>
DEV void epilogue(const GemmParams& p, int m, int n, float v0, float v1, float v2, float v3) {
  if constexpr (EPI == EPI_F32) {
    float* C = reinterpret_cast<float*>(p.C) + (size_t)blockIdx.z * p.slab_stride;
    *reinterpret_cast<float4*>(C + (size_t)m * p.ldc + n) = make_float4(v0, v1, v2, v3);
  } else {
    if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
      const float4 b = *reinterpret_cast<const float4*>(p.bias + n);
      v0 += b.x; v1 += b.y; v2 += b.z; v3 += b.w;
    }
    if constexpr (EPI == EPI_BIAS_GELU) {
      // GELU on the bf16-rounded pre-activation, exactly what the backward re-reads.
      const uint2 u = make_uint2(pack_bf2(v0, v1), pack_bf2(v2, v3));
      *reinterpret_cast<uint2*>(p.aux + (size_t)m * p.ldaux + n) = u;
      v0 = gelu_erf(lo_bf(u.x)); v1 = gelu_erf(hi_bf(u.x));
      v2 = gelu_erf(lo_bf(u.y)); v3 = gelu_erf(hi_bf(u.y));
    }
    if constexpr (EPI == EPI_GELU_BWD) {
      const uint2 u = *reinterpret_cast<const uint2*>(p.aux + (size_t)m * p.ldaux + n);
      v0 *= gelu_erf_grad(lo_bf(u.x)); v1 *= gelu_erf_grad(hi_bf(u.x));
      v2 *= gelu_erf_grad(lo_bf(u.y)); v3 *= gelu_erf_grad(hi_bf(u.y));
    }
    if constexpr (EPI == EPI_ADD) {
      const uint2 r = *reinterpret_cast<const uint2*>(p.res + (size_t)m * p.ldres + n);
      v0 += lo_bf(r.x); v1 += hi_bf(r.x); v2 += lo_bf(r.y); v3 += hi_bf(r.y);
    }
    bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
    *reinterpret_cast<uint2*>(C + (size_t)m * p.ldc + n) = make_uint2(pack_bf2(v0, v1), pack_bf2(v2, v3));
  }
}

template <int BM, int BN, bool AK, bool BKM, int EPI, int WM = 2, int WN = 2>
__global__ __launch_bounds__(64 * WM * WN, 8 / (WM * WN) > 0 ? 8 / (WM * WN) : 1) void gemm_kernel(GemmParams p) {
  constexpr int NW = WM * WN;
  using OA = Operand<BM, AK, BKT, NW>;
  using OB = Operand<BN, BKM, BKT, NW>;
  constexpr int TM = BM / WM, TN = BN / WN;  // per-wave tile
  constexpr int MI = TM / 16, NI = TN / 16;  // 16x16 sub-tiles per wave
  constexpr int BUF = OA::BYTES + OB::BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;

  // Tile walk: M-major inside each N column panel so consecutive logical tiles
  // share the B (weight) panel; XCD remap keeps those on one L2.
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = p.N / BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  int tm, tn;
  tile_coords(bid, tiles_m, tiles_n, p.group_m, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.z * p.k_split;
  const int nk = p.k_split / BKT;

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  OA::stage(p.A, p.lda, m0, kbeg, p.M, smem, wid, lane);
  OB::stage(p.B, p.ldb, n0, kbeg, p.N, smem + OA::BYTES, wid, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * BUF;
    if (kt + 1 < nk && !(p.diag & 1)) {
      char* nxt = smem + ((kt + 1) & 1) * BUF;
      OA::stage(p.A, p.lda, m0, kbeg + (kt + 1) * BKT, p.M, nxt, wid, lane);
      OB::stage(p.B, p.ldb, n0, kbeg + (kt + 1) * BKT, p.N, nxt + OA::BYTES, wid, lane);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = OA::frag(cur, wr * TM + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) bfr[j] = OB::frag(cur + OA::BYTES, wc * TN + j * 16, s, lane);
      if (p.diag & 2) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j) acc[i][j][0] += (float)(af[i][0] ^ bfr[j][1]);
        continue;
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (p.diag & 4) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) t += acc[i][j][0] + acc[i][j][3];
    if (t != 1234.5f) return;
  }

  // ---------------------------------------------------------------- epilogue
  // lane owns C[m][n..n+3] of every sub-tile (operand-swapped MFMA).
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = m0 + wr * TM + i * 16 + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = n0 + wc * TN + j * 16 + 4 * (lane >> 4);
      float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
      epilogue<EPI>(p, m, n, v0, v1, v2, v3);
    }
  }
}

template <int N>
DEV void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Counted wait for "all but the youngest n*L LDS-DMA ops" (n = stages still allowed in flight).
template <int L, int MAXN>
DEV void wait_stages(int n) {
  if constexpr (MAXN >= 3) { if (n >= 3) { wait_vm<3 * L>(); return; } }
  if constexpr (MAXN >= 2) { if (n >= 2) { wait_vm<2 * L>(); return; } }
  if constexpr (MAXN >= 1) { if (n >= 1) { wait_vm<L>(); return; } }
  wait_vm<0>();
}

// Multi-stage ring variant: STAGES LDS buffers, tile t+STAGES-1's DMA issued while
// tile t is consumed; a counted vmcnt (never 0 in steady state) + ONE raw s_barrier
// per K tile keeps STAGES-2 tiles in flight across the barrier
// (cdna_hip_programming.md "Pipelining across barriers").
template <int BM, int BN, int BK, int STAGES, bool AK, bool BKM, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_pipe_kernel(GemmParams p) {
  using OA = Operand<BM, AK, BK>;
  using OB = Operand<BN, BKM, BK>;
  constexpr int MI = BM / 32, NI = BN / 32;
  constexpr int BUF = OA::BYTES + OB::BYTES;
  constexpr int L = OA::PER_WAVE + OB::PER_WAVE;  // DMA ops per wave per stage
  constexpr int SUB = BK / 32;                     // 32-deep MFMA steps per tile
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = p.N / BN;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  int tm, tn;
  tile_coords(bid, tiles_m, tiles_n, p.group_m, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.z * p.k_split;
  const int nk = p.k_split / BK;

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int t) {
    char* b = smem + (t % STAGES) * BUF;
    OA::stage(p.A, p.lda, m0, kbeg + t * BK, p.M, b, wid, lane);
    OB::stage(p.B, p.ldb, n0, kbeg + t * BK, p.N, b + OA::BYTES, wid, lane);
  };
#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (t < nk) issue(t);

  for (int t = 0; t < nk; ++t) {
    const int ahead = min(STAGES - 2, nk - 1 - t);  // younger stages allowed in flight
    wait_stages<L, STAGES - 2>(ahead);
    __builtin_amdgcn_s_barrier();
    if (t + STAGES - 1 < nk) issue(t + STAGES - 1);
    const char* cur = smem + (t % STAGES) * BUF;
#pragma unroll
    for (int s = 0; s < SUB; ++s) {
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = OA::frag(cur, wr * (BM / 2) + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) bfr[j] = OB::frag(cur + OA::BYTES, wc * (BN / 2) + j * 16, s, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  }

#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = m0 + wr * (BM / 2) + i * 16 + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = n0 + wc * (BN / 2) + j * 16 + 4 * (lane >> 4);
      float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
      epilogue<EPI>(p, m, n, v0, v1, v2, v3);
    }
  }
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

// Kernel variants (FD_GEMM_VARIANT env for A/B benchmarking; default picks per kind):
//   0: 2-stage ring, BK=64        1: 4-stage ring, BK=32
//   2: 3-stage ring, BK=64        3: 3-stage ring, BK=32
int variant_override() {
  static int v = [] {
    const char* e = getenv("FD_GEMM_VARIANT");
    return e ? atoi(e) : -1;
  }();
  return v;
}

template <int BM, int BN, bool AK, bool BKM, int EPI>
void launch(const GemmParams& p, int splits, hipStream_t st, int variant) {
  const dim3 grid(((p.M + BM - 1) / BM) * (p.N / BN), 1, splits);
  switch (variant) {
    case 1: hipLaunchKernelGGL((gemm_pipe_kernel<BM, BN, 32, 4, AK, BKM, EPI>), grid, dim3(256), 0, st, p); break;
    case 2: hipLaunchKernelGGL((gemm_pipe_kernel<BM, BN, 64, 3, AK, BKM, EPI>), grid, dim3(256), 0, st, p); break;
    case 3: hipLaunchKernelGGL((gemm_pipe_kernel<BM, BN, 32, 3, AK, BKM, EPI>), grid, dim3(256), 0, st, p); break;
    default: hipLaunchKernelGGL((gemm_kernel<BM, BN, AK, BKM, EPI>), grid, dim3(256), 0, st, p); break;
  }
}

// Pick BN in {128, 96, 64} maximising (wave-quantisation efficiency x tile efficiency)
// on 256 CUs x 2 resident blocks.
int pick_bn(int M, int N, bool allow96) {
  const int cand[3] = {128, 96, 64};
  const double tile_eff[3] = {1.0, 0.93, 0.84};
  const int slots = 512;
  int best = 64;
  double best_s = -1;
  for (int c = 0; c < 3; ++c) {
    const int bn = cand[c];
    if (N % bn != 0 || (bn == 96 && !allow96)) continue;
    const long tiles = (long)((M + 127) / 128) * (N / bn);
    const long rounds = (tiles + slots - 1) / slots;
    const double q = (double)tiles / (double)(rounds * slots);
    const double s = q * tile_eff[c];
    if (s > best_s) { best_s = s; best = bn; }
  }
  return best;
}

// Tile configurations of the 2-stage kernel (FD_GEMM_TILE=<id> forces one):
//   0: 128x128 (2x2 waves)  1: 128x96 (2x2, K-major B only)  2: 128x64 (2x2)
//   3: 256x128 (4x2)        4: 256x192 (4x2, K-major B only) 5: 256x64 (4x2)
int tile_override() {
  static int v = [] {
    const char* e = getenv("FD_GEMM_TILE");
    return e ? atoi(e) : -1;
  }();
  return v;
}

template <bool AK, bool BKM, int EPI>
bool launch_tile(const GemmParams& p, int tile, int splits, hipStream_t st) {
  auto grid = [&](int bm, int bn) { return dim3(((p.M + bm - 1) / bm) * (p.N / bn), 1, splits); };
  switch (tile) {
    case 0: if (p.N % 128) return false;
      hipLaunchKernelGGL((gemm_kernel<128, 128, AK, BKM, EPI>), grid(128, 128), dim3(256), 0, st, p); return true;
    case 1: if constexpr (BKM) { if (p.N % 96) return false;
      hipLaunchKernelGGL((gemm_kernel<128, 96, AK, BKM, EPI>), grid(128, 96), dim3(256), 0, st, p); return true; }
      return false;
    case 2: if (p.N % 64) return false;
      hipLaunchKernelGGL((gemm_kernel<128, 64, AK, BKM, EPI>), grid(128, 64), dim3(256), 0, st, p); return true;
    case 3: if constexpr (AK) { if (p.N % 128) return false;
      hipLaunchKernelGGL((gemm_kernel<256, 128, AK, BKM, EPI, 4, 2>), grid(256, 128), dim3(512), 0, st, p); return true; }
      return false;
    case 4: if constexpr (BKM && AK) { if (p.N % 192) return false;
      hipLaunchKernelGGL((gemm_kernel<256, 192, AK, BKM, EPI, 4, 2>), grid(256, 192), dim3(512), 0, st, p); return true; }
      return false;
    case 5: if constexpr (AK) { if (p.N % 64) return false;
      hipLaunchKernelGGL((gemm_kernel<256, 64, AK, BKM, EPI, 4, 2>), grid(256, 64), dim3(512), 0, st, p); return true; }
      return false;
  }
  return false;
}

// BN = 96 only exists for the 2-stage BK=64 kernel (96-row tiles do not split into
// whole 1 KiB DMA pieces per wave at BK=32).
template <bool AK, bool BKM, int EPI>
void dispatch(const GemmParams& p, int bn, int splits, hipStream_t st, int variant) {
  const int to = tile_override();
  if (to >= 0 && variant == 0 && launch_tile<AK, BKM, EPI>(p, to, splits, st)) return;
  if constexpr (BKM) {
    if (bn == 96 && variant == 0) {
      const dim3 grid(((p.M + 127) / 128) * (p.N / 96), 1, splits);
      hipLaunchKernelGGL((gemm_kernel<128, 96, AK, BKM, EPI>), grid, dim3(256), 0, st, p);
      return;
    }
  }
  if (bn == 128) launch<128, 128, AK, BKM, EPI>(p, splits, st, variant);
  else launch<128, 64, AK, BKM, EPI>(p, splits, st, variant);
}

}  // namespace

// ---------------------------------------------------------------- C ABI
extern "C" {

// kind: 0 = NT (y = x W^T), 1 = NN (dx = dy W), 2 = TN (dW = dy^T x, fp32 out)
// Returns 0 on success, nonzero on unsupported shape.
int fd_gemm(int kind, int epi, const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
            const float* bias, void* aux, int ldaux, const void* res, int ldres, float* workspace,
            long long workspace_elems, int accumulate, hipStream_t st) {
  if (K % BKT != 0 || N % 64 != 0 || M <= 0) return 1;
  GemmParams p{};
  p.A = (const bf16_t*)A; p.B = (const bf16_t*)B; p.C = C;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.bias = bias; p.aux = (bf16_t*)aux; p.ldaux = ldaux; p.res = (const bf16_t*)res; p.ldres = ldres;
  p.k_split = K;
  {
    static const int diag = [] { const char* e = getenv("FD_GEMM_DIAG"); return e ? atoi(e) : 0; }();
    p.diag = diag;
  }
  // Group height: A-panels of gm x 128 rows x K (bf16) should take ~half of a 4 MiB L2.
  {
    const long long panel = 128ll * K * 2;
    int gm = (int)std::max(1ll, std::min(16ll, (2ll << 20) / panel));
    const char* e = getenv("FD_GEMM_GROUP_M");
    if (e) gm = atoi(e);
    p.group_m = gm;
  }
  const int ov = variant_override();
  if (kind == 0) {
    const int var = ov >= 0 ? ov : 0;
    // Measured on MI355X (scripts/gemm_bench.py, FD_GEMM_TILE sweep): 128x64 tiles win
    // for the DistilBERT forward shapes except the wide FFN1 (N = 3072), where the
    // 8-wave 256x192 tile does (one round of 256 tiles at M = 4096).
    if (var == 0 && tile_override() < 0) {
      const int tile = (N % 192 == 0 && N >= 3072 && M >= 2048) ? 4 : 2;
      bool ok = false;
      switch (epi) {
        case EPI_BIAS: ok = launch_tile<true, true, EPI_BIAS>(p, tile, 1, st); break;
        case EPI_BIAS_GELU: ok = launch_tile<true, true, EPI_BIAS_GELU>(p, tile, 1, st); break;
        case EPI_BF16: ok = launch_tile<true, true, EPI_BF16>(p, tile, 1, st); break;
        default: return 2;
      }
      if (ok) return 0;
    }
    const int bn = pick_bn(M, N, var == 0);
    switch (epi) {
      case EPI_BIAS: dispatch<true, true, EPI_BIAS>(p, bn, 1, st, var); break;
      case EPI_BIAS_GELU: dispatch<true, true, EPI_BIAS_GELU>(p, bn, 1, st, var); break;
      case EPI_BF16: dispatch<true, true, EPI_BF16>(p, bn, 1, st, var); break;
      default: return 2;
    }
    return 0;
  }
  if (kind == 1) {
    const int var = ov >= 0 ? ov : 0;
    const int bn = pick_bn(M, N, false);
    switch (epi) {
      case EPI_BF16: dispatch<true, false, EPI_BF16>(p, bn, 1, st, var); break;
      case EPI_GELU_BWD: dispatch<true, false, EPI_GELU_BWD>(p, bn, 1, st, var); break;
      case EPI_ADD: dispatch<true, false, EPI_ADD>(p, bn, 1, st, var); break;
      default: return 2;
    }
    return 0;
  }
  if (kind == 2) {
    // dW[M=out][N=in] fp32.  Split K (the token dim) until the grid covers the
    // chip; slabs go to `workspace` and are reduced deterministically.
    if (M % 128 != 0) return 3;
    const int var = ov >= 0 ? ov : 0;
    // Measured: 128x64 for dW of out_lin / lin1 / lin2, 128x128 for the fused QKV dW.
    const int bn = (N % 128 == 0 && M > 1024 && M < 3072 && N < 3072) ? 128 : 64;
    const int tiles = (M / 128) * (N / bn);
    int splits = 1;
    while (tiles * splits < 384 && (K / (splits * 2)) % BKT == 0 && K / (splits * 2) >= 512) splits *= 2;
    const long long slab = (long long)M * N;
    if (splits > 1 && workspace_elems < slab * splits) splits = 1;
    p.k_split = K / splits;
    float* out = (float*)C;
    if (splits == 1 && !accumulate) {
      p.slab_stride = 0;
      dispatch<false, false, EPI_F32>(p, bn, 1, st, var);
      return 0;
    }
    if (ldc != N) return 4;
    p.C = workspace; p.ldc = N; p.slab_stride = slab;
    dispatch<false, false, EPI_F32>(p, bn, splits, st, var);
    const long long n4 = slab / 4;
    const int blocks = (int)std::min<long long>((n4 + 255) / 256, 2048);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, workspace, out, n4, slab, splits,
                       accumulate);
    return 0;
  }
  return 5;
}

}  // extern "C"
