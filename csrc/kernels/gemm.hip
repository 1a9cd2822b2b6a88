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
// Design (MI355X-first, see cdna_hip_programming.md §5):
//  * 256 threads = 4 waves in a 2x2 grid; each wave owns a (BM/2)x(BN/2) tile of
//    16x16 MFMA sub-tiles; K step 64 (two 32-deep MFMA steps).
//  * Register-staged, double-buffered LDS: the next K tile's 16-byte global loads
//    are issued before the current tile's MFMAs and written to the other LDS
//    buffer after them (T14) -> one barrier per K tile.
//  * K-major operands live in LDS as [rows][64] with a 16-byte-chunk XOR swizzle
//    (chunk ^= (row>>1)&7) so the ds_read_b128 fragment reads are conflict-free.
//    MN-major operands live as [64 k-rows][BM] and are read with the gfx950
//    transposing ds_read_b64_tr_b16 (T10); their chunk swizzle (fk) makes the
//    two 16-lane groups of each half-wave hit disjoint banks.
//  * Operands are swapped inside the MFMA (D = B^T A^T = C^T) so each lane ends
//    up owning 4 consecutive output columns: 8-byte bf16 / 16-byte fp32 stores,
//    and bias / residual / GELU-aux loads are vectorised the same way.
//  * XCD-aware bijective block remap (T1) + M-major tile walk for L2 reuse.
#include "common.h"
#include <algorithm>

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
};

constexpr int BKT = 64;

// Swizzle of 16-byte chunks for the MN-major ([k][mn]) LDS image.
template <int BMN>
DEV int fk(int k) {
  if constexpr (BMN == 128) return ((k & 3) | ((k >> 1) & 4)) << 1;
  else return (((k >> 1) & 1) | ((k >> 2) & 2)) << 1;
}

template <int ROWS, bool KMAJ>
struct Operand {
  // bytes of one LDS buffer
  static constexpr int BYTES = ROWS * BKT * 2;
  static constexpr int LOADS = ROWS * BKT / 8 / 256;  // 16-byte loads per thread
  static constexpr int CHUNKS = KMAJ ? 8 : ROWS / 8;  // 16-byte chunks per LDS row
  static constexpr int ROWB = KMAJ ? 128 : ROWS * 2;  // LDS row bytes

  // Global -> registers for K tile starting at k0; rows beyond `lim` read as 0
  // (K-major only: the token dimension of activations).
  DEV static void gload(uint4 (&r)[LOADS], const bf16_t* base, int ld, int row0, int k0, int lim,
                        int tid) {
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int id = i * 256 + tid;
      if constexpr (KMAJ) {
        const int rr = id >> 3, c = id & 7;
        if (row0 + rr < lim)
          r[i] = *reinterpret_cast<const uint4*>(base + (size_t)(row0 + rr) * ld + k0 + c * 8);
        else
          r[i] = make_uint4(0, 0, 0, 0);
      } else {
        const int kk = id / CHUNKS, c = id % CHUNKS;
        r[i] = *reinterpret_cast<const uint4*>(base + (size_t)(k0 + kk) * ld + row0 + c * 8);
      }
    }
  }

  DEV static void lstore(const uint4 (&r)[LOADS], char* lds, int tid) {
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int id = i * 256 + tid;
      int off;
      if constexpr (KMAJ) {
        const int rr = id >> 3, c = id & 7;
        off = rr * 128 + ((c ^ ((rr >> 1) & 7)) << 4);
      } else {
        const int kk = id / CHUNKS, c = id % CHUNKS;
        off = kk * ROWB + ((c ^ fk<ROWS>(kk)) << 4);
      }
      *reinterpret_cast<uint4*>(lds + off) = r[i];
    }
  }

  // MFMA fragment for rows [row0, row0+16) and k-step s (32 deep).
  DEV static bf16x8 frag(const char* lds, int row0, int s, int lane) {
    if constexpr (KMAJ) {
      const int row = row0 + (lane & 15);
      const int c = s * 4 + (lane >> 4);
      return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
    } else {
      const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
      const int c = (row0 >> 3) + (p >> 1);
      bf16x8 out;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = s * 32 + 8 * g + 4 * h + q;
        const char* addr = lds + k * ROWB + ((c ^ fk<ROWS>(k)) << 4) + (p & 1) * 8;
        bf16x4v v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) bf16x4v*)(addr));
        out[4 * h + 0] = v[0];
        out[4 * h + 1] = v[1];
        out[4 * h + 2] = v[2];
        out[4 * h + 3] = v[3];
      }
      return out;
    }
  }
};

template <int BM, int BN, bool AK, bool BKM, int EPI>
__global__ __launch_bounds__(256) void gemm_kernel(GemmParams p) {
  using OA = Operand<BM, AK>;
  using OB = Operand<BN, BKM>;
  constexpr int MI = BM / 32, NI = BN / 32;  // 16x16 sub-tiles per wave
  __shared__ __attribute__((aligned(16))) char smem[2 * (OA::BYTES + OB::BYTES)];
  char* const sa0 = smem;
  char* const sb0 = smem + 2 * OA::BYTES;
#define SA(b) (sa0 + (b) * OA::BYTES)
#define SB(b) (sb0 + (b) * OB::BYTES)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  // Tile walk: M-major inside each N column panel so consecutive logical tiles
  // share the B (weight) panel; XCD remap keeps those on one L2.
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = p.N / BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid % tiles_m, tn = bid / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.z * p.k_split;
  const int nk = p.k_split / BKT;

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[OA::LOADS], rb[OB::LOADS];
  OA::gload(ra, p.A, p.lda, m0, kbeg, p.M, tid);
  OB::gload(rb, p.B, p.ldb, n0, kbeg, p.N, tid);
  OA::lstore(ra, SA(0), tid);
  OB::lstore(rb, SB(0), tid);
  __syncthreads();

  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      OA::gload(ra, p.A, p.lda, m0, kbeg + (kt + 1) * BKT, p.M, tid);
      OB::gload(rb, p.B, p.ldb, n0, kbeg + (kt + 1) * BKT, p.N, tid);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = OA::frag(SA(buf), wr * (BM / 2) + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) bfr[j] = OB::frag(SB(buf), wc * (BN / 2) + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
    }
    if (more) {
      OA::lstore(ra, SA(buf ^ 1), tid);
      OB::lstore(rb, SB(buf ^ 1), tid);
    }
    __syncthreads();
    buf ^= 1;
  }

#undef SA
#undef SB
  // ---------------------------------------------------------------- epilogue
  // lane owns C[m][n..n+3] of every sub-tile (operand-swapped MFMA).
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = m0 + wr * (BM / 2) + i * 16 + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = n0 + wc * (BN / 2) + j * 16 + 4 * (lane >> 4);
      float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
      if constexpr (EPI == EPI_F32) {
        float* C = reinterpret_cast<float*>(p.C) + (size_t)blockIdx.z * p.slab_stride;
        *reinterpret_cast<float4*>(C + (size_t)m * p.ldc + n) = make_float4(v0, v1, v2, v3);
      } else {
        if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
          const float4 b = *reinterpret_cast<const float4*>(p.bias + n);
          v0 += b.x; v1 += b.y; v2 += b.z; v3 += b.w;
        }
        if constexpr (EPI == EPI_BIAS_GELU) {
          *reinterpret_cast<uint2*>(p.aux + (size_t)m * p.ldaux + n) =
              make_uint2(pack_bf2(v0, v1), pack_bf2(v2, v3));
          // GELU on the bf16-rounded pre-activation, exactly what the backward
          // will see when it re-reads aux.
          const uint2 u = make_uint2(pack_bf2(v0, v1), pack_bf2(v2, v3));
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
        *reinterpret_cast<uint2*>(C + (size_t)m * p.ldc + n) =
            make_uint2(pack_bf2(v0, v1), pack_bf2(v2, v3));
      }
    }
  }
}

// out[i] = (accumulate ? out[i] : 0) + sum_z slab[z][i]   (deterministic split-K reduce)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slabs,
                                                            float* __restrict__ out, long long n4,
                                                            long long stride, int splits,
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

template <int BM, int BN, bool AK, bool BKM, int EPI>
void launch(const GemmParams& p, int splits, hipStream_t st) {
  const int tiles = ((p.M + BM - 1) / BM) * (p.N / BN);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, AK, BKM, EPI>), dim3(tiles, 1, splits), dim3(256), 0, st,
                     p);
}

}  // namespace

// ---------------------------------------------------------------- C ABI
extern "C" {

// kind: 0 = NT (y = x W^T), 1 = NN (dx = dy W), 2 = TN (dW = dy^T x, fp32 out)
// Returns 0 on success, nonzero on unsupported shape.
int fd_gemm(int kind, int epi, const void* A, const void* B, void* C, int M, int N, int K, int lda,
            int ldb, int ldc, const float* bias, void* aux, int ldaux, const void* res, int ldres,
            float* workspace, long long workspace_elems, int accumulate, hipStream_t st) {
  if (K % BKT != 0 || N % 64 != 0) return 1;
  GemmParams p{};
  p.A = (const bf16_t*)A; p.B = (const bf16_t*)B; p.C = C;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.bias = bias; p.aux = (bf16_t*)aux; p.ldaux = ldaux; p.res = (const bf16_t*)res; p.ldres = ldres;
  p.k_split = K;
  const bool wide = (N % 128 == 0) && ((long long)((M + 127) / 128) * (N / 128) >= 512);
  if (kind == 0) {
    if (epi == EPI_BIAS) {
      if (wide) launch<128, 128, true, true, EPI_BIAS>(p, 1, st);
      else launch<128, 64, true, true, EPI_BIAS>(p, 1, st);
    } else if (epi == EPI_BIAS_GELU) {
      if (wide) launch<128, 128, true, true, EPI_BIAS_GELU>(p, 1, st);
      else launch<128, 64, true, true, EPI_BIAS_GELU>(p, 1, st);
    } else if (epi == EPI_BF16) {
      if (wide) launch<128, 128, true, true, EPI_BF16>(p, 1, st);
      else launch<128, 64, true, true, EPI_BF16>(p, 1, st);
    } else return 2;
    return 0;
  }
  if (kind == 1) {
    if (epi == EPI_BF16) {
      if (wide) launch<128, 128, true, false, EPI_BF16>(p, 1, st);
      else launch<128, 64, true, false, EPI_BF16>(p, 1, st);
    } else if (epi == EPI_GELU_BWD) {
      if (wide) launch<128, 128, true, false, EPI_GELU_BWD>(p, 1, st);
      else launch<128, 64, true, false, EPI_GELU_BWD>(p, 1, st);
    } else if (epi == EPI_ADD) {
      if (wide) launch<128, 128, true, false, EPI_ADD>(p, 1, st);
      else launch<128, 64, true, false, EPI_ADD>(p, 1, st);
    } else return 2;
    return 0;
  }
  if (kind == 2) {
    // dW[M=out][N=in] fp32.  Split K (the token dim) until the grid covers the
    // chip ~2x; slabs go to `workspace` and are reduced deterministically.
    if (M % 128 != 0) return 3;
    const int tiles = (M / 128) * (N / 128 > 0 && N % 128 == 0 ? N / 128 : N / 64);
    const bool n128 = N % 128 == 0;
    int splits = 1;
    while (tiles * splits < 512 && (K / (splits * 2)) % BKT == 0 && K / (splits * 2) >= 256) splits *= 2;
    const long long slab = (long long)M * N;
    if (splits > 1 && workspace_elems < slab * splits) splits = 1;
    p.k_split = K / splits;
    float* out = (float*)C;
    if (splits == 1 && !accumulate) {
      p.slab_stride = 0;
      if (n128) launch<128, 128, false, false, EPI_F32>(p, 1, st);
      else launch<128, 64, false, false, EPI_F32>(p, 1, st);
      return 0;
    }
    p.C = workspace; p.ldc = N; p.slab_stride = slab;
    if (n128) launch<128, 128, false, false, EPI_F32>(p, splits, st);
    else launch<128, 64, false, false, EPI_F32>(p, splits, st);
    if (ldc != N) return 4;
    const long long n4 = slab / 4;
    const int blocks = (int)std::min<long long>((n4 + 255) / 256, 2048);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, workspace, out, n4, slab,
                       splits, accumulate);
    return 0;
  }
  return 5;
}

}  // extern "C"
