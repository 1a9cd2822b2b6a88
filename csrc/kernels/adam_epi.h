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
