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
// C[M][N] (+)= A^T B with A [K][M], B [K][N] bf16 (same K for every problem).  p != nullptr:
// apply Adam to the finished gradient tile (state laid out like C) instead of storing it.
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
};
