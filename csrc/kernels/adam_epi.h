// Adam state of one weight matrix, laid out like its gradient (row-major [M][N]).
// Handed to the weight-gradient GEMM (gemm.hip) so its epilogue applies the
// optimizer step to the finished fp32 gradient tile instead of storing it: the
// gradient never round-trips through HBM and the Adam traffic (p, m, v, bf16
// shadow) streams while other tiles of the same grid are still on the MFMAs.
// Plain C types: included by the kernels and by the host binding.
#pragma once
#include <stdint.h>

struct FdAdamEpi {
  float* p;           // fp32 master (nullptr = no fused optimizer)
  float* m;           // first moment
  float* v;           // second moment
  uint16_t* sh;       // bf16 compute shadow (nullable)
  const int* step;    // device step counter (already advanced for this step)
  float lr, b1, b2, eps, wd;
  int decoupled;      // AdamW-style decay
};

// One weight-gradient problem of the all-layer launch (gemm.hip gemm_dw_batch_kernel):
// C[M][N] (+)= A^T B with A [K][M], B [K][N] bf16 (K: this problem's rows, a multiple of 64 --
// the pruned last block's problems run on the padded [CLS] rows only).  p != nullptr: apply Adam
// to the finished gradient tile (state laid out like C) instead of storing it.
struct FdDwProb {
  const uint16_t* A;
  const uint16_t* B;
  float* C;
  float* p;
  float* m;
  float* v;
  uint16_t* sh;       // bf16 shadow (nullable)
  int M, N;
  int tile0;          // filled by the launcher
  int accumulate;
  int K;              // rows of A and B (0: the launch's K)
  // nullable: also bias[m] (+)= sum_k A[k][m] -- the producer's bias gradient (the qkv bias: A is
  // dqkv), summed by the tiles of the first column block while their K loops read A anyway
  float* bias;
  int half;           // filled by the launcher: 1 = tiled 256 x 128 (the mixed schedule's tail class)
};

// The rest of the optimizer step, run by extra blocks of the all-layer dW launch beside its last
// tiles (gemm.hip dwb_rest) instead of two launches of its own after it: every parameter the fused
// epilogues do not update.  p / g / m / v / sh are the whole arenas; runs: the run table over them
// ([start4, count4, prefix4] rows, head_optim.hip AdamArgs) of everything but the word table, n4
// its float4 total; the word table ([wrows][wrow4 float4] at element woff) by its row flags
// (ever: has Adam state, now: has a gradient this step; weight decay 0).  The qkv bias, whose
// gradient the launch itself sums, is updated by the tiles that sum it (GemmParams::acol_*).
struct FdAdamRest {
  float* p;
  const float* g;
  float* m;
  float* v;
  uint16_t* sh;
  const long long* runs;
  long long n4;
  int nruns;
  int wrows, wrow4;
  long long woff;
  const unsigned char* ever;
  const unsigned char* now;
  int flat_blocks, row_blocks;  // filled by the launcher
  int first;                    // the rest blocks lead the grid (else they follow the tiles)
};

#define FD_LN_XSITES 128

// LayerNorm fused into an N = hidden GEMM (gemm.hip gemm_ln_kernel).  The column tiles of one
// row block exchange per-row partial statistics through tagged granules in `stats`, so every
// tile normalises its own slice from its accumulators.
//   forward  (out_lin + sa_layer_norm, lin2 + output_layer_norm):
//     z = dropout(acc + bias) + res  (bf16, kept for the backward);  C = LN(z) * gamma + beta
//   backward (the dX GEMM that produces the LN output gradient dy = acc + res):
//     C = dz = rstd * (gamma dy - mean(gamma dy) - xhat mean(gamma dy xhat)),  xhat from z;
//     dx = dropout'(dz) (the producer's output gradient);  per-row-block column partials of
//     dgamma = sum dy xhat, dbeta = sum dy, dbias = sum dx into colpart[tiles_m][3][N].
struct FdLnEpi {
  const float* gamma;
  const float* beta;      // forward only
  float* mean;            // [M] forward: out; backward: in
  float* rstd;
  uint16_t* z;            // [M][N] bf16 pre-LN sum: forward out (nullable), backward in
  uint16_t* dx;           // backward: dropout-masked gradient (nullable without dropout)
  float* colpart;         // backward: [tiles_m][3][N]
  uint64_t* stats;        // [tiles_m][tiles_n][2][BM] {tag, value} granules (forward mean / M2,
                          // backward s1 / s2 per row); zeroed once
  int* cnt;               // [1]: exchange epoch, advanced once per model forward (norm.hip
                          // emb_fwd_kernel) or by the caller (ops/kernels.py ln_epoch_advance)
  int* err;               // set nonzero if a row-block rendezvous timed out (fatal: the host
                          // raises at its next check, ops/kernels.py check_ln_error)
  uint32_t xsite;         // exchange call site, unique per LN launch between two epoch advances
                          // (< FD_LN_XSITES): granule tag = epoch * FD_LN_XSITES + xsite + 1
  const uint32_t* seed_ptr;
  uint32_t site, thr;     // dropout (thr == 0: none), hashed like norm.hip's ln kernels
  float dscale;
  const int* row_map;     // packed row -> padded row (dropout hash only; nullable)
  float eps;
  // two-K-half tiles (gemm.hip gemm_ln2_kernel): the two blocks of a 128 x 128 product tile trade
  // the fp32 column halves they do not finish -- xbuf [pairs][2][32 KiB] and xflag [pairs][2]
  // {tag, 1} granules (the stats buffer's tail: zeroed with it at an epoch wrap).  Nullable.
  float* xbuf;
  uint64_t* xflag;
  // Next-launch operand prefetch (nullable): while waiting for the row statistics each block
  // touches its 1/grid slice of pf (one load per 64 bytes), so the next GEMM finds its weight in
  // MALL / L2 instead of HBM.  The loaded values are dead.
  const char* pf;
  long long pf_bytes;
};

// The pruned training step's head fused into the split-K LayerNorm epilogue of the last block's
// output LayerNorm (splitk.hip sk_ln_kernel, FD_HEAD_IN_SK): row m's block, after writing y[m],
// computes the head logits / loss / dlogits of [CLS] row m (< B), the head gradient of y[m] and the
// LayerNorm backward of the row (the unit-seeded loss's gradient), and leaves per-row partials of
// the head dW / db, the loss mean and the LayerNorm affine gradients for the deferred column sums.
struct FdSkHead {
  const float* W;          // [2][N] head weight (fp32 master)
  const float* bias;       // [2]
  const long long* labels; // [B]
  const float* tlogits;    // [B][2] teacher logits (nullable: plain cross-entropy)
  float kd_T, kd_alpha;
  const uint32_t* seed_ptr;  // head dropout (hashed like head_common.h)
  uint32_t site, thr;
  float dscale;
  int B;
  const int* own;          // [B + 1] packed sequence starts (nullable): empty sequences get no dh
  float* logits;           // [B][2]
  float* dlogits;          // [B][2]
  uint16_t* dz;            // [M][N] bf16 LayerNorm input gradient
  uint16_t* dx;            // [M][N] bf16 dropout-masked (nullable without dropout)
  float* colpart;          // [M][3][N] dgamma / dbeta / dbias rows
  float* hpart;            // [M][2][N] head dW rows
  float* dbpart;           // [M][2] head db rows
  float* lpart;            // [M] row loss / B
  float* loss;             // [1] the batch loss: sum of lpart, written by the launch's last row block
  unsigned* ticket;        // [1] row blocks done, ever (zeroed once, never reset)
};

