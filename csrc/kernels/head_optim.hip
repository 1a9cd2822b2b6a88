// Classifier head + CE loss, eval metrics, Adam/AdamW and FedAvg helpers (gfx950).
//
// Head (client1.py:57-64, :108): pooled = hidden[:, 0, :] -> Dropout(0.3) ->
// Linear(768, 2) -> CrossEntropy(mean).  B <= 1024 rows; one 256-thread block,
// fixed reduction order (deterministic).  2-class CE == BCE-with-logits on z1-z0.
//
// Adam (client1.py:380, torch.optim.Adam defaults, bias-corrected): one launch
// over the whole flat fp32 parameter arena (66,364,418 params) with float4
// loads, writing the fp32 master, m, v and the bf16 compute shadow in the same
// pass.  The step count and the dropout seed counter live on the device so the
// whole train step can be replayed as a HIP graph.
//
// Eval metrics (client1.py:134-142): per-batch mean CE added to a device
// accumulator, correct / TP / FP / FN / TN counts and P(class 1) -- replacing
// the reference's four host syncs per eval batch.
#include "common.h"

#include <cstdlib>

namespace {

#include "head_common.h"

// One wave per batch row (grid = ceil(B/4) blocks): logits only (no labels), or the rows of a
// batch too large for head_fwd_mean_kernel (their loss reduced by head_loss_mean_kernel).
__global__ __launch_bounds__(256) void head_fwd_kernel(HeadArgs a) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b < a.B) head_row(a, b, threadIdx.x & 63);
}

__global__ __launch_bounds__(64) void head_loss_mean_kernel(HeadArgs a) { loss_mean(a, threadIdx.x); }

// With labels and B <= HEAD_MEAN_MAXB: ONE block of 16 waves takes every row (wave w: rows w,
// w + 16, ...), then its first wave reduces the row losses -- the same sums in the same order as
// head_fwd_kernel + head_loss_mean_kernel, one launch instead of two.
constexpr int HEAD_MEAN_MAXB = 1024;
__global__ __launch_bounds__(1024) void head_fwd_mean_kernel(HeadArgs a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int b = w; b < a.B; b += 32) {  // rows b and b + 16 of this wave, loads interleaved
    const int rows[2] = {b, b + 16 < a.B ? b + 16 : -1};
    float z0[2], z1[2];
    head_logits_n<2>(a, rows, lane, z0, z1);
#pragma unroll
    for (int r = 0; r < 2; ++r)
      if (rows[r] >= 0) head_row_out(a, rows[r], lane, z0[r], z1[r]);
  }
  __syncthreads();  // (every row loss written; workgroup-visible)
  if (w == 0) loss_mean(a, lane);
}

// Is `row` the [CLS] row of some non-empty sequence (the rows the compute blocks write)?
DEV bool is_cls_row(const HeadArgs& a, int row) {
  if (!a.cls) return row % a.S == 0 && row / a.S < a.B;
  int lo = 0, hi = a.B;  // cls = sequence starts: non-decreasing; first b with cls_row(b) > row
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int)cls_row(a, mid) <= row) lo = mid + 1;
    else hi = mid;
  }
  const int b = lo - 1;  // the last sequence claiming `row` (duplicates: the later one owns it)
  return b >= 0 && (int)cls_row(a, b) == row && !empty_seq(a, b);
}

// Blocks [0, ceil(D/256)): dW / db and the [CLS] rows of dhidden.  Blocks beyond: zero every
// other row of dhidden (so the caller needs no separate fill launch).
// Column blocks: 32 columns x 8 row groups per 256-thread block (D / 32 blocks), so every
// thread has at most ceil(B / 8) [CLS] rows to load -- all issued before any use -- instead of
// a serial walk over the batch; the 8 group partials of dW are summed through LDS in a fixed
// order (deterministic).  The remaining blocks zero the non-[CLS] rows of dhidden.
constexpr int HB_COLS = 32, HB_GROUPS = 8, HB_ROWS = 8;  // rows per thread held in flight (B <= 64)
__global__ __launch_bounds__(256) void head_bwd_kernel(HeadArgs a) {
  const int nc = (a.D + HB_COLS - 1) / HB_COLS;
  if ((int)blockIdx.x >= nc) {
    const int per_row = a.D / 8;  // uint4 chunks
    const long long total = (long long)a.T * per_row;
    for (long long i = (long long)(blockIdx.x - nc) * 256 + threadIdx.x; i < total;
         i += (long long)(gridDim.x - nc) * 256) {
      const int row = (int)(i / per_row);
      if (!is_cls_row(a, row)) reinterpret_cast<uint4*>(a.dhidden)[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    return;
  }
  __shared__ float red[2][HB_GROUPS][HB_COLS];
  const int c = threadIdx.x % HB_COLS, grp = threadIdx.x / HB_COLS;
  const int col = blockIdx.x * HB_COLS + c;
  const bool live = col < a.D;
  const int colc = live ? col : 0;
  const bool drop = a.thr != 0;
  const uint32_t seed = drop ? hash32(a.seed_ptr[0], a.site) : 0u;
  const float gs = a.gscale ? a.gscale[0] : 1.f;
  const float w0 = a.W[colc], w1 = a.W[a.D + colc];
  float g0 = 0.f, g1 = 0.f;
  for (int b0 = grp; b0 < a.B; b0 += HB_GROUPS * HB_ROWS) {
    float x[HB_ROWS];
    size_t row[HB_ROWS];
#pragma unroll
    for (int u = 0; u < HB_ROWS; ++u) {  // every row's load in flight before the first use
      const int b = min(b0 + u * HB_GROUPS, a.B - 1);
      row[u] = cls_row(a, b);
      x[u] = bf2f(a.hidden[row[u] * a.D + colc]);
    }
#pragma unroll
    for (int u = 0; u < HB_ROWS; ++u) {
      const int b = b0 + u * HB_GROUPS;
      if (b >= a.B) break;
      const float d0 = a.dlog_in[2 * b] * gs, d1 = a.dlog_in[2 * b + 1] * gs;
      const bool keep = !drop || drop_keep(seed, (uint32_t)(b * a.D + colc), a.thr);
      const float sc = drop ? (keep ? a.dscale : 0.f) : 1.f;
      const float xv = x[u] * sc;
      head_col_acc(g0, d0, xv);
      head_col_acc(g1, d1, xv);
      // an empty sequence shares its [CLS] row with the next one: the later sequence writes it
      const bool last_owner = b + 1 >= a.B || cls_row(a, b + 1) != row[u];
      if (live && last_owner && !empty_seq(a, b)) a.dhidden[row[u] * a.D + col] = (bf16_t)head_dh(d0, d1, w0, w1, sc);
    }
  }
  red[0][grp][c] = g0;
  red[1][grp][c] = g1;
  __syncthreads();
  if (grp < 2 && live) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < HB_GROUPS; ++i) s += red[grp][i][c];
    float* dst = a.dW + grp * a.D + col;
    *dst = a.accumulate ? *dst + s : s;
  }
  if (blockIdx.x == 0 && threadIdx.x < 2) {
    float s = 0.f;
    for (int b = 0; b < a.B; ++b) s += a.dlog_in[2 * b + threadIdx.x] * gs;
    a.db[threadIdx.x] = a.accumulate ? a.db[threadIdx.x] + s : s;
  }
}

// acc: [0] = sum of per-batch mean loss (double), counts: [0] correct [1] tp [2] fp [3] fn [4] tn
__global__ __launch_bounds__(256) void eval_metrics_kernel(const float* logits, const long long* labels, int B,
                                                           double* acc, long long* counts, float* prob1,
                                                           long long* preds) {
  __shared__ float sl[256];
  __shared__ int sc[5][256];
  const int t = threadIdx.x;
  float l = 0.f;
  int c[5] = {0, 0, 0, 0, 0};
  for (int b = t; b < B; b += 256) {
    const float z0 = logits[2 * b], z1 = logits[2 * b + 1];
    const float mx = fmaxf(z0, z1);
    const float lse = mx + logf(expf(z0 - mx) + expf(z1 - mx));
    const int y = (int)labels[b];
    l += lse - (y ? z1 : z0);
    const int pred = z1 > z0 ? 1 : 0;  // torch.max picks the first index on ties
    if (prob1) prob1[b] = expf(z1 - lse);
    if (preds) preds[b] = pred;
    c[0] += pred == y;
    c[1] += pred == 1 && y == 1;
    c[2] += pred == 1 && y == 0;
    c[3] += pred == 0 && y == 1;
    c[4] += pred == 0 && y == 0;
  }
  sl[t] = l;
  for (int k = 0; k < 5; ++k) sc[k][t] = c[k];
  __syncthreads();
  if (t == 0) {
    float s = 0.f;
    long long cc[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 256; ++i) {
      s += sl[i];
      for (int k = 0; k < 5; ++k) cc[k] += sc[k][i];
    }
    acc[0] += (double)(s / B);
    for (int k = 0; k < 5; ++k) counts[k] += cc[k];
  }
}

#include "adam_common.h"

template <bool NT, bool NTP = false>
__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
  float step_size, inv_sqrt_bc2;
  adam_bias_corr(a.step, a.lr, a.b1, a.b2, step_size, inv_sqrt_bc2);
  for (long long vi = blockIdx.x * 256ll + threadIdx.x; vi < a.n4; vi += (long long)gridDim.x * 256)
    adam_flat4<NT, NTP>(a, vi, step_size, inv_sqrt_bc2);
}

// Adam over the rows of a table that have state (ever[row] != 0; weight decay 0): one wave per
// row, which leaves at once unless the row is flagged, so every flagged row is updated in
// parallel (row_len / 4 float4 per row, gradient 0 unless now[row]) with adam_kernel's
// arithmetic (adam_math4: bitwise the dense launch's result).  The word-embedding table: ~30 k
// rows, a few hundred of which a CICIDS2017 run ever touches; the dense launch walked all 23 M
// parameters.
__global__ __launch_bounds__(256) void adam_rows_kernel(AdamArgs a, int rows, int row4) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows || !a.touched[row]) return;  // wave-uniform
  float step_size, inv_sqrt_bc2;
  adam_bias_corr(a.step, a.lr, a.b1, a.b2, step_size, inv_sqrt_bc2);
  if (row4 == 192) adam_row768(a, row, lane, step_size, inv_sqrt_bc2);
  else adam_row(a, 0, row, row4, lane, step_size, inv_sqrt_bc2);
}

__global__ void step_kernel(int* step, uint32_t* seed) {
  if (step) step[0] += 1;
  if (seed) seed[0] += 1;
}

// p *= scale (optional) and shadow = bf16(p): FedAvg finalisation / shadow refresh.
__global__ __launch_bounds__(256) void scale_cast_kernel(float* p, bf16_t* shadow, long long n4, float scale) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float4 v = reinterpret_cast<float4*>(p)[i];
    if (scale != 1.f) {
      v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
      reinterpret_cast<float4*>(p)[i] = v;
    }
    if (shadow) reinterpret_cast<uint2*>(shadow)[i] = make_uint2(pack_bf2(v.x, v.y), pack_bf2(v.z, v.w));
  }
}

// dst = a * x + b * y over fp32 arenas (sample-weighted FedAvg pre-scale / blends).
__global__ __launch_bounds__(256) void axpby_kernel(float* dst, const float* x, const float* y, float a, float b,
                                                    long long n4) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const float4 u = reinterpret_cast<const float4*>(x)[i];
    float4 r = make_float4(a * u.x, a * u.y, a * u.z, a * u.w);
    if (y) {
      const float4 w = reinterpret_cast<const float4*>(y)[i];
      r.x += b * w.x; r.y += b * w.y; r.z += b * w.z; r.w += b * w.w;
    }
    reinterpret_cast<float4*>(dst)[i] = r;
  }
}

int grid_for(long long n4) { return (int)std::min<long long>((n4 + 255) / 256, 4096); }

}  // namespace

extern "C" {

int fd_head_fwd(const void* hidden, int B, int S, int D, const float* W, const float* bias,
                const uint32_t* seed_ptr, uint32_t site, uint32_t thr, float dscale, const long long* labels,
                float* logits, float* loss, float* dlogits, float* row_loss, const int* cls, int T,
                const float* tlogits, float kd_T, float kd_alpha, float* loss_acc, hipStream_t st) {
  if (B > 65536) return 1;
  if (tlogits && (!labels || !(kd_T > 0.f))) return 3;
  HeadArgs a{};
  a.tlogits = tlogits; a.kd_T = kd_T; a.kd_alpha = kd_alpha;
  a.cls = cls; a.T = T;
  a.hidden = (const bf16_t*)hidden; a.B = B; a.S = S; a.D = D; a.W = W; a.bias = bias;
  a.seed_ptr = seed_ptr; a.site = site; a.thr = thr; a.dscale = dscale; a.labels = labels;
  a.logits = logits; a.loss = loss; a.dlogits = dlogits; a.row_loss = row_loss;
  a.loss_acc = labels ? loss_acc : nullptr;
  if (labels && !row_loss) return 2;
  if (labels && B <= HEAD_MEAN_MAXB) {
    hipLaunchKernelGGL(head_fwd_mean_kernel, dim3(1), dim3(1024), 0, st, a);
    return 0;
  }
  hipLaunchKernelGGL(head_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, st, a);
  if (labels) hipLaunchKernelGGL(head_loss_mean_kernel, dim3(1), dim3(64), 0, st, a);
  return 0;
}

int fd_head_bwd(const void* hidden, int B, int S, int D, const float* W, const uint32_t* seed_ptr, uint32_t site,
                uint32_t thr, float dscale, const float* dlogits, float* dW, float* db, void* dhidden,
                int accumulate, const int* cls, int T, const float* gscale, const int* own, hipStream_t st) {
  HeadArgs a{};
  a.gscale = gscale;
  a.cls = cls; a.T = T; a.own = own;
  a.hidden = (const bf16_t*)hidden; a.B = B; a.S = S; a.D = D; a.W = W;
  a.seed_ptr = seed_ptr; a.site = site; a.thr = thr; a.dscale = dscale; a.dlog_in = dlogits;
  a.dW = dW; a.db = db; a.dhidden = (bf16_t*)dhidden; a.accumulate = accumulate;
  if (D % 8) return 1;
  // compute blocks + zeroing blocks (~4 uint4 stores per thread over the non-[CLS] rows)
  const long long chunks = (long long)T * (D / 8);
  const int zb = (int)std::min<long long>((chunks + 1023) / 1024, 1024);
  hipLaunchKernelGGL(head_bwd_kernel, dim3((D + HB_COLS - 1) / HB_COLS + zb), dim3(256), 0, st, a);
  return 0;
}

int fd_eval_metrics(const float* logits, const long long* labels, int B, double* acc, long long* counts,
                    float* prob1, long long* preds, hipStream_t st) {
  hipLaunchKernelGGL(eval_metrics_kernel, dim3(1), dim3(256), 0, st, logits, labels, B, acc, counts, prob1, preds);
  return 0;
}

int fd_adam(float* p, const float* g, float* m, float* v, void* shadow, long long n, const int* step, float lr,
            float b1, float b2, float eps, float wd, int decoupled, const unsigned char* touched,
            const unsigned char* now, long long skip_off, long long skip_rows, int row_len, const long long* runs,
            int nruns, long long run_total4, hipStream_t st) {
  if (n % 4 != 0 || skip_off % 4 != 0 || row_len % 4 != 0) return 1;
  if (wd != 0.f && touched) return 3;  // skipping untouched rows is exact only without weight decay
  if (runs && (nruns <= 0 || run_total4 <= 0)) return 4;
  AdamArgs a{p, g, m, v, (bf16_t*)shadow, runs ? run_total4 : n / 4, step, lr, b1, b2, eps, wd, decoupled,
             skip_off / 4, (skip_off + skip_rows * row_len) / 4, row_len / 4, touched, now, runs, nruns};
  const int grid = grid_for(n / 4);
  // FD_ADAM_NT: 0 = default cache policy, 1 = nontemporal g/m/v, 2 = also the fp32 master (default:
  // 2.336 vs 2.366-2.387 ms/step, profiles/r1_ab_adam_nt_master.txt -- only the bf16 shadow is re-read soon)
  static const int nt = [] { const char* e = getenv("FD_ADAM_NT"); return e ? atoi(e) : 2; }();
  if (nt == 2)
    hipLaunchKernelGGL((adam_kernel<true, true>), dim3(grid), dim3(256), 0, st, a);
  else if (nt)
    hipLaunchKernelGGL((adam_kernel<true, false>), dim3(grid), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((adam_kernel<false, false>), dim3(grid), dim3(256), 0, st, a);
  return 0;
}

// Adam over the flagged rows of a [rows][row_len] table (weight decay 0; see adam_rows_kernel).
int fd_adam_rows(float* p, const float* g, float* m, float* v, void* shadow, int rows, int row_len, const int* step,
                 float lr, float b1, float b2, float eps, const unsigned char* ever, const unsigned char* now,
                 hipStream_t st) {
  if (row_len % 4 != 0 || rows <= 0 || !ever) return 1;
  AdamArgs a{p, g, m, v, (bf16_t*)shadow, 0, step, lr, b1, b2, eps, 0.f, 0, 0, 0, row_len / 4, ever, now, nullptr, 0};
  hipLaunchKernelGGL(adam_rows_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, a, rows, row_len / 4);  // wave per row
  return 0;
}

int fd_step(int* step, uint32_t* seed, hipStream_t st) {
  hipLaunchKernelGGL(step_kernel, dim3(1), dim3(1), 0, st, step, seed);
  return 0;
}

int fd_scale_cast(float* p, void* shadow, long long n, float scale, hipStream_t st) {
  if (n % 4 != 0) return 1;
  hipLaunchKernelGGL(scale_cast_kernel, dim3(grid_for(n / 4)), dim3(256), 0, st, p, (bf16_t*)shadow, n / 4, scale);
  return 0;
}

int fd_axpby(float* dst, const float* x, const float* y, float a, float b, long long n, hipStream_t st) {
  if (n % 4 != 0) return 1;
  hipLaunchKernelGGL(axpby_kernel, dim3(grid_for(n / 4)), dim3(256), 0, st, dst, x, y, a, b, n / 4);
  return 0;
}

}  // extern "C"
