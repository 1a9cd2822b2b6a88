// Host-only sanitizer harness for the launch-validation layer (csrc/binding.cpp).
//
// The binding is the only thing between Python and a hand-written kernel's grid: it must
// reject every call whose shapes the kernel does not support, and pass every pointer with
// the extent the kernel will touch.  Here it is compiled with g++ -fsanitize=address,undefined
// against CPU ATen (FD_HOST_VALIDATION), with the fd_* launchers replaced by stubs that
// (a) count calls and (b) check that every region the real kernel would read or write --
// derived from the launch arguments exactly as the kernel derives it -- lies inside a buffer
// the test registered.  The driver then makes valid calls (no exception, no violation) and
// invalid ones (a c10::Error, and NO launcher call).  Run by tests/test_host_sanitizers.py.
#define FD_HOST_VALIDATION 1
#include <algorithm>
#include "../binding.cpp"

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace hc {
struct Region { uintptr_t lo, hi; };
std::vector<Region> regions;
std::vector<std::string> violations;
int calls = 0;

void reg(const at::Tensor& t) {
  const uintptr_t p = reinterpret_cast<uintptr_t>(t.data_ptr());
  regions.push_back({p, p + (uintptr_t)(t.numel() * t.element_size())});
}
void span(const void* p, long long bytes, const char* what) {
  if (bytes <= 0) return;
  if (!p) { violations.push_back(std::string("null ") + what); return; }
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p), hi = lo + (uintptr_t)bytes;
  for (const Region& r : regions)
    if (lo >= r.lo && hi <= r.hi) return;
  violations.push_back(std::string("out of bounds: ") + what + " (" + std::to_string(bytes) + " B)");
}
void opt_span(const void* p, long long bytes, const char* what) { if (p) span(p, bytes, what); }
}  // namespace hc

// ------------------------------------------------------------------ stub launchers
extern "C" {
const void* g_hc_pf = nullptr;
long long g_hc_pf_bytes = 0;
int fd_gemm_pf(const void* pf, long long bytes) {
  g_hc_pf = pf;
  g_hc_pf_bytes = pf ? bytes : 0;
  return 0;
}
int fd_gemm_ex(int kind, int epi, const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
               int ldc, const float* bias, void* aux, int ldaux, const void* res, int ldres, float* workspace,
               long long workspace_elems, int accumulate, const FdAdamEpi* adam,
               float* colsum, int* colsum_blocks, void* aux_out, hipStream_t) {
  ++hc::calls;
  if (g_hc_pf) hc::span(g_hc_pf, g_hc_pf_bytes, "gemm prefetch");  // (the launch's one-shot prefetch)
  g_hc_pf = nullptr;
  g_hc_pf_bytes = 0;
  if (kind == 0) {  // A [M][lda] (K used), B [N][ldb], C [M][ldc] bf16
    hc::span(A, ((long long)(M - 1) * lda + K) * 2, "gemm A");
    hc::span(B, ((long long)(N - 1) * ldb + K) * 2, "gemm B");
  } else if (kind == 1) {  // A [M][lda], B [K][ldb] (N used)
    hc::span(A, ((long long)(M - 1) * lda + K) * 2, "gemm A");
    hc::span(B, ((long long)(K - 1) * ldb + N) * 2, "gemm B");
  } else {  // A [K][lda] (M used), B [K][ldb]
    hc::span(A, ((long long)(K - 1) * lda + M) * 2, "gemm A");
    hc::span(B, ((long long)(K - 1) * ldb + N) * 2, "gemm B");
  }
  hc::span(C, ((long long)(M - 1) * ldc + N) * (kind == 2 ? 4 : 2), "gemm C");
  if (epi == 1 || epi == 2) hc::span(bias, (long long)N * 4, "gemm bias");
  // (epi 2: u is optional -- the kernel writes it only when given)
  if (epi == 3 || (epi == 2 && aux)) hc::span(aux, ((long long)(M - 1) * ldaux + N) * 2, "gemm aux");
  if (epi == 4) hc::span(res, ((long long)(M - 1) * ldres + N) * 2, "gemm res");
  if (aux_out) hc::span(aux_out, ((long long)(M - 1) * ldaux + N) * 2, "gemm aux_out");
  if (colsum && colsum_blocks) {
    *colsum_blocks = (M + 127) / 128;
    hc::span(colsum, (long long)*colsum_blocks * N * 4, "gemm colsum");
  }
  if (kind == 2 && workspace_elems > 0) hc::span(workspace, workspace_elems * 4, "gemm workspace");
  if (adam && adam->p) {
    hc::span(adam->p, (long long)M * N * 4, "adam p");
    hc::span(adam->m, (long long)M * N * 4, "adam m");
    hc::span(adam->v, (long long)M * N * 4, "adam v");
    hc::opt_span(adam->sh, (long long)M * N * 2, "adam shadow");
  }
  (void)accumulate;
  return 0;
}
int fd_gemm(int kind, int epi, const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
            const float* bias, void* aux, int ldaux, const void* res, int ldres, float* workspace,
            long long workspace_elems, int accumulate, const FdAdamEpi* adam,
            float* colsum, int* colsum_blocks, hipStream_t st) {
  return fd_gemm_ex(kind, epi, A, B, C, M, N, K, lda, ldb, ldc, bias, aux, ldaux, res, ldres, workspace,
                    workspace_elems, accumulate, adam, colsum, colsum_blocks, nullptr, st);
}
int fd_gemm_set_cfg(int, int, int) { return 0; }
int fd_gemm_stamps(unsigned long long*, int) { return -1; }
int fd_attn_stamps(unsigned long long*, int) { return -1; }
int fd_attn_set_split(int) { return 0; }
int fd_gemm_dw2(const void* A0, const void* B0, float* C0, int M0, int N0, const void* A1, const void* B1, float* C1,
                int M1, int N1, int K, float* workspace, long long workspace_elems, int,
                const FdAdamEpi* adams, int, int* splits_out, hipStream_t) {
  ++hc::calls;
  hc::span(A0, (long long)K * M0 * 2, "dw2 A0");
  hc::span(B0, (long long)K * N0 * 2, "dw2 B0");
  hc::span(C0, (long long)M0 * N0 * 4, "dw2 C0");
  hc::span(A1, (long long)K * M1 * 2, "dw2 A1");
  hc::span(B1, (long long)K * N1 * 2, "dw2 B1");
  hc::span(C1, (long long)M1 * N1 * 4, "dw2 C1");
  hc::opt_span(workspace, workspace_elems * 4, "dw2 workspace");
  (void)adams;
  if (splits_out) *splits_out = 0;
  return 0;
}
int fd_gemm_dw2_splits(int, int, int, int, int) { return 1; }
int fd_gemm_dw_batch(int n, const FdDwProb* probs, int K, const int* step, const float* hyper, int cfg,
                     const FdAdamRest* rest, hipStream_t) {
  ++hc::calls;
  if (rest) {
    if (!hyper || !step) hc::violations.push_back("dw_batch rest without the fused Adam");
    if (rest->runs) hc::span(rest->runs, (long long)rest->nruns * 3 * 8, "dw_batch rest runs");
    if (rest->ever) {
      hc::span(rest->ever, rest->wrows, "dw_batch rest ever");
      hc::span(rest->now, rest->wrows, "dw_batch rest now");
      hc::span(rest->p + rest->woff, (long long)rest->wrows * rest->wrow4 * 16, "dw_batch rest word rows");
    }
  }
  if (n <= 0 || n > 32) hc::violations.push_back("dw_batch: problem count");
  for (int i = 0; i < n; ++i) {
    const FdDwProb& q = probs[i];
    const long long mn = (long long)q.M * q.N;
    const long long Kq = q.K > 0 ? q.K : K;
    if (Kq % 64) hc::violations.push_back("dw_batch: K % 64");
    hc::span(q.A, Kq * q.M * 2, "dw_batch A");
    hc::span(q.B, Kq * q.N * 2, "dw_batch B");
    hc::opt_span(q.bias, (long long)q.M * 4, "dw_batch bias");
    if (q.p) {
      hc::span(q.p, mn * 4, "dw_batch adam p");
      hc::span(q.m, mn * 4, "dw_batch adam m");
      hc::span(q.v, mn * 4, "dw_batch adam v");
      hc::opt_span(q.sh, mn * 2, "dw_batch adam shadow");
      hc::span(step, 4, "dw_batch step");
      if (!hyper) hc::violations.push_back("dw_batch: fused Adam without hyper-parameters");
    } else {
      hc::span(q.C, mn * 4, "dw_batch C");
    }
  }
  (void)cfg;
  return 0;
}
int fd_adam_rows(float* p, const float* g, float* m, float* v, void* shadow, int rows, int row_len, const int* step,
                 float, float, float, float, const unsigned char* ever, const unsigned char* now, hipStream_t) {
  ++hc::calls;
  const long long n = (long long)rows * row_len;
  hc::span(p, n * 4, "adam_rows p");
  hc::span(g, n * 4, "adam_rows g");
  hc::span(m, n * 4, "adam_rows m");
  hc::span(v, n * 4, "adam_rows v");
  hc::opt_span(shadow, n * 2, "adam_rows shadow");
  hc::span(step, 4, "adam_rows step");
  hc::span(ever, rows, "adam_rows ever");
  hc::opt_span(now, rows, "adam_rows now");
  return 0;
}
int fd_gemm_splitk(int epi, const void* A, const void* Bt, int M, int N, int K, float* workspace,
                   long long workspace_elems, int splits, const float* bias, void* C, void* aux, void* aux_out,
                   const void* res, float* colsum, int* colsum_blocks, const FdLnEpi* ln, const FdSkHead* hd,
                   int b_mn, hipStream_t) {
  ++hc::calls;
  (void)b_mn;  // (W [K][N] or W^T [N][K]: the same N * K elements)
  const long long mn = (long long)M * N;
  if (hd && hd->W) {  // the fused head (FdSkHead): B rows of head outputs, M rows of partials
    hc::span(hd->W, (long long)2 * N * 4, "splitk head W");
    hc::span(hd->labels, (long long)hd->B * 8, "splitk head labels");
    hc::span(hd->logits, (long long)hd->B * 8, "splitk head logits");
    hc::span(hd->dlogits, (long long)hd->B * 8, "splitk head dlogits");
    hc::span(hd->dz, mn * 2, "splitk head dz");
    hc::opt_span(hd->dx, mn * 2, "splitk head dx");
    hc::span(hd->colpart, mn * 3 * 4, "splitk head colpart");
    hc::span(hd->hpart, mn * 2 * 4, "splitk head hpart");
    hc::span(hd->dbpart, (long long)M * 8, "splitk head dbpart");
    hc::span(hd->lpart, (long long)M * 4, "splitk head lpart");
    hc::span(hd->loss, 4, "splitk head loss");
    hc::span(hd->ticket, 4, "splitk head ticket");
    hc::opt_span(hd->own, (long long)(hd->B + 1) * 4, "splitk head own");
  }
  if (splits <= 0) splits = 1;
  hc::span(A, (long long)M * K * 2, "splitk A");
  hc::span(Bt, (long long)N * K * 2, "splitk Bt");
  hc::span(C, mn * 2, "splitk C");
  hc::span(workspace, std::min(workspace_elems, (long long)splits * mn) * 4, "splitk workspace");
  if (epi == 1 || epi == 2 || epi == 6) hc::span(bias, (long long)N * 4, "splitk bias");
  if (epi == 2 || epi == 3) hc::span(aux, mn * 2, "splitk aux");
  hc::opt_span(aux_out, mn * 2, "splitk aux_out");
  if (epi == 4 || epi >= 6) hc::span(res, mn * 2, "splitk res");
  if (colsum) {
    if (colsum_blocks) *colsum_blocks = (M + 31) / 32;
    hc::span(colsum, (long long)((M + 31) / 32) * N * 4, "splitk colsum");
  }
  if (ln) {
    hc::span(ln->gamma, (long long)N * 4, "splitk gamma");
    hc::span(ln->mean, (long long)M * 4, "splitk mean");
    hc::span(ln->rstd, (long long)M * 4, "splitk rstd");
    if (epi == 7) {
      hc::span(ln->z, mn * 2, "splitk z");
      hc::span(ln->colpart, mn * 3 * 4, "splitk colpart");
      if (ln->thr) hc::span(ln->dx, mn * 2, "splitk dx");
    } else {
      hc::span(ln->beta, (long long)N * 4, "splitk beta");
      hc::opt_span(ln->z, mn * 2, "splitk z");
    }
    if (ln->thr) {
      hc::span(ln->seed_ptr, 4, "splitk seed");
      hc::opt_span(ln->row_map, (long long)M * 4, "splitk row_map");
    }
  }
  return splits;
}
int fd_gemm_ln(int bwd, const void* A, const void* Bt, void* C, int M, int N, int K, const float* bias,
               const void* res, int ldres, const FdLnEpi* ln, int cfg, int b_mn, hipStream_t) {
  ++hc::calls;
  (void)b_mn;  // (W [K][N] or W^T [N][K]: the same N * K elements)
  const int bm = cfg == 13 ? 64 : 128;
  const long long tm = (M + bm - 1) / bm, mn = (long long)M * N;
  hc::span(A, (long long)M * K * 2, "gemm_ln A");
  hc::span(Bt, (long long)N * K * 2, "gemm_ln Bt");
  hc::span(C, mn * 2, "gemm_ln C");
  hc::span(res, (long long)M * ldres * 2, "gemm_ln res");
  hc::span(ln->gamma, (long long)N * 4, "gemm_ln gamma");
  hc::span(ln->mean, (long long)M * 4, "gemm_ln mean");
  hc::span(ln->rstd, (long long)M * 4, "gemm_ln rstd");
  hc::span(ln->stats, tm * (N / 64) * 2 * bm * 8, "gemm_ln stats");
  hc::span(ln->cnt, 4, "gemm_ln cnt");
  hc::span(ln->err, 4, "gemm_ln err");
  if (ln->pf) hc::span(ln->pf, ln->pf_bytes, "gemm_ln prefetch");  // (loads one dword per 64 B inside it)
  if (ln->xbuf) {  // two-K-half tiles: pairs x 2 x 32 (128-row) / 64 KiB (256-row) of partials,
                   // pairs x 2 flag granules; the 256-row tiles' statistics rows
    const long long pairs = tm * (N / 128), tm256 = (M + 255) / 256;
    hc::span(ln->xbuf, std::max(pairs * 2 * 32768, tm256 * (N / 128) * 2 * 65536), "gemm_ln xbuf");
    hc::span(ln->xflag, pairs * 2 * 8, "gemm_ln xflag");
    hc::span(ln->stats, tm256 * (N / 64) * 2 * 256 * 8, "gemm_ln stats (256-row tiles)");
  }
  if (bwd) {
    hc::span(ln->z, mn * 2, "gemm_ln z");
    hc::span(ln->colpart, tm * 3 * N * 4, "gemm_ln colpart");
    if (ln->thr) hc::span(ln->dx, mn * 2, "gemm_ln dx");
  } else {
    hc::span(bias, (long long)N * 4, "gemm_ln bias");
    hc::span(ln->beta, (long long)N * 4, "gemm_ln beta");
    hc::opt_span(ln->z, mn * 2, "gemm_ln z");
  }
  if (ln->thr) {
    hc::span(ln->seed_ptr, 4, "gemm_ln seed");
    hc::opt_span(ln->row_map, (long long)M * 4, "gemm_ln row_map");
  }
  return (int)tm;
}
int fd_splitk_reduce_batched(int n, const float* const* slabs, float* const* outs, const long long* numel,
                             const int* splits, const int*, hipStream_t) {
  ++hc::calls;
  for (int i = 0; i < n; ++i) {
    hc::span(slabs[i], numel[i] * splits[i] * 4, "reduce slabs");
    hc::span(outs[i], numel[i] * 4, "reduce out");
  }
  return 0;
}
const char* fd_comm_last_error() { return ""; }
int fd_comm_load(const char*) { return 0; }
int fd_comm_unique_id_bytes() { return 128; }
int fd_comm_get_unique_id(void*) { return 0; }
int fd_comm_init(void**, int, int, const void*) { return 0; }
int fd_comm_destroy(void*) { return 0; }
int fd_comm_async_error(void*) { return 0; }
int fd_comm_wait(void*, hipStream_t, long long) { return 0; }
int fd_comm_abort(void*) { return 0; }
int fd_comm_allreduce(void*, const void*, void*, long long, int, int, hipStream_t) { return 0; }
int fd_comm_broadcast(void*, void*, long long, int, int, hipStream_t) { return 0; }
int fd_comm_allgather(void*, const void*, void*, long long, int, hipStream_t) { return 0; }
int fd_attn_fwd(const void* qkv, const float* kbias, void* ctx, float* lse, int B, int S, int H, const uint32_t* seed,
                uint32_t, uint32_t, float, const int* cu, int rows, uint64_t* dmask, int, void* cxc, void* xc,
                const void* xres, int Bp, int, hipStream_t) {
  ++hc::calls;
  const long long D = (long long)H * 64;
  hc::opt_span(cxc, (long long)Bp * D * 2, "attn cxc");
  hc::opt_span(xc, (long long)Bp * D * 2, "attn xc");
  hc::opt_span(xres, rows * D * 2, "attn xres");
  hc::opt_span(dmask, (long long)B * H * 256 * 8, "attn dmask");
  hc::span(qkv, rows * 3 * D * 2, "attn qkv");
  hc::span(ctx, rows * D * 2, "attn ctx");
  hc::span(lse, (long long)B * H * S * 4, "attn lse");
  hc::span(seed, 4, "attn seed");
  if (cu) hc::span(cu, (long long)(B + 1) * 4, "attn cu");
  else hc::span(kbias, (long long)B * S * 4, "attn kbias");
  return 0;
}
int fd_gemm_attn_fwd(const void* x, const void* w, const float* bias, void* qkv, int M, int K, const float* kbias,
                     void* ctx, float* lse, int B, int S, int H, const uint32_t* seed, uint32_t, uint32_t, float,
                     const int* cu, int rows, uint64_t* dmask, int, void* cxc, void* xc, const void* xres, int Bp,
                     uint64_t* flags, int nflags, const int* cnt, int, int* err, int, int, hipStream_t) {
  ++hc::calls;
  if (g_hc_pf) hc::span(g_hc_pf, g_hc_pf_bytes, "gemm_attn prefetch");
  g_hc_pf = nullptr;
  g_hc_pf_bytes = 0;
  const long long D = (long long)H * 64, N = 3 * D;
  hc::span(x, (long long)M * K * 2, "gemm_attn x");
  hc::span(w, N * K * 2, "gemm_attn w");
  hc::span(bias, N * 4, "gemm_attn bias");
  hc::span(qkv, (long long)M * N * 2, "gemm_attn qkv");
  const long long tiles = ((M + 127) / 128) * (N / 192);
  if (tiles > nflags) hc::violations.push_back("gemm_attn: more tiles than flags");
  hc::span(flags, tiles * 8, "gemm_attn flags");
  hc::span(cnt, 4, "gemm_attn cnt");
  hc::span(err, 4, "gemm_attn err");
  hc::opt_span(cxc, (long long)Bp * D * 2, "gemm_attn cxc");
  hc::opt_span(xc, (long long)Bp * D * 2, "gemm_attn xc");
  hc::opt_span(xres, rows * D * 2, "gemm_attn xres");
  hc::opt_span(dmask, (long long)B * H * 256 * 8, "gemm_attn dmask");
  hc::span(ctx, rows * D * 2, "gemm_attn ctx");
  hc::span(lse, (long long)B * H * S * 4, "gemm_attn lse");
  hc::span(seed, 4, "gemm_attn seed");
  if (cu) hc::span(cu, (long long)(B + 1) * 4, "gemm_attn cu");
  else hc::span(kbias, (long long)B * S * 4, "gemm_attn kbias");
  return 0;
}
int fd_attn_bwd_proj(const void* qkv, const float* kbias, const void* ctx, const float* lse, const void* dy,
                     const void* w, int M, int K, int, void* dqkv, int B, int S, int H, const uint32_t* seed,
                     uint32_t, uint32_t, float, const int* cu, int rows, const uint64_t* dmask, const void* dresc,
                     void* dres, int, hipStream_t) {
  ++hc::calls;
  const long long D = (long long)H * 64;
  hc::opt_span(dmask, (long long)B * H * 256 * 8, "attn bwd proj dmask");
  hc::span(qkv, rows * 3 * D * 2, "attn bwd proj qkv");
  hc::span(dqkv, rows * 3 * D * 2, "attn bwd proj dqkv");
  hc::span(ctx, rows * D * 2, "attn bwd proj ctx");
  hc::span(dy, (long long)M * K * 2, "attn bwd proj dy");
  hc::span(w, (long long)K * D * 2, "attn bwd proj w");
  hc::opt_span(dresc, (long long)M * D * 2, "attn bwd proj dresc");
  hc::opt_span(dres, rows * D * 2, "attn bwd proj dres");
  hc::span(lse, (long long)B * H * S * 4, "attn bwd proj lse");
  hc::span(seed, 4, "attn bwd proj seed");
  if (cu) hc::span(cu, (long long)(B + 1) * 4, "attn bwd proj cu");
  else hc::span(kbias, (long long)B * S * 4, "attn bwd proj kbias");
  return 0;
}
int fd_attn_bwd(const void* qkv, const float* kbias, const void* ctx, const float* lse, const void* dctx, float* delta,
                void* dqkv, int B, int S, int H, const uint32_t* seed, uint32_t, uint32_t, float, const int* cu,
                int rows, const uint64_t* dmask, int, const void* dresc, void* dres, int, hipStream_t) {
  ++hc::calls;
  const long long D = (long long)H * 64;
  hc::opt_span(dmask, (long long)B * H * 256 * 8, "attn bwd dmask");
  hc::span(qkv, rows * 3 * D * 2, "attn bwd qkv");
  hc::span(dqkv, rows * 3 * D * 2, "attn bwd dqkv");
  hc::span(ctx, rows * D * 2, "attn bwd ctx");
  // (compact [CLS] gradients: dctx / dresc hold >= B rows, dres the full layout)
  hc::span(dctx, (dres ? B : rows) * D * 2, "attn bwd dctx");
  hc::opt_span(dresc, (long long)B * D * 2, "attn bwd dresc");
  hc::opt_span(dres, rows * D * 2, "attn bwd dres");
  hc::span(lse, (long long)B * H * S * 4, "attn bwd lse");
  hc::span(delta, (long long)B * H * S * 4, "attn bwd delta");
  hc::span(seed, 4, "attn bwd seed");
  if (cu) hc::span(cu, (long long)(B + 1) * 4, "attn bwd cu");
  else hc::span(kbias, (long long)B * S * 4, "attn bwd kbias");
  return 0;
}
int fd_mask_to_bias(const void*, int, float*, long, hipStream_t) { ++hc::calls; return 0; }
int fd_ln_fwd(const void* x, const void* r, const float* gamma, const float* beta, void* y, float* mean, float* rstd,
              int T, int D, float, const uint32_t* seed, uint32_t, uint32_t, float, const int* row_map, hipStream_t) {
  ++hc::calls;
  const long long n = (long long)T * D;
  hc::span(x, n * 2, "ln x");
  hc::opt_span(r, n * 2, "ln r");
  hc::span(y, n * 2, "ln y");
  hc::span(gamma, (long long)D * 4, "ln gamma");
  hc::span(beta, (long long)D * 4, "ln beta");
  hc::span(mean, (long long)T * 4, "ln mean");
  hc::span(rstd, (long long)T * 4, "ln rstd");
  hc::span(seed, 4, "ln seed");
  hc::opt_span(row_map, (long long)T * 4, "ln row_map");
  return 0;
}
int fd_ln_bwd(const void* dy, const void* x, const void* r, const float* gamma, const float* mean, const float* rstd,
              void* dz, void* dx, float* dgamma, float* dbeta, float* dbias, float* work, int T, int D,
              const uint32_t* seed, uint32_t, uint32_t, float, int, const int* row_map, int, int* nblk_out,
              int, hipStream_t) {
  ++hc::calls;
  const long long n = (long long)T * D;
  hc::span(dy, n * 2, "ln bwd dy");
  hc::span(x, n * 2, "ln bwd x");
  hc::opt_span(r, n * 2, "ln bwd r");
  hc::span(dz, n * 2, "ln bwd dz");
  hc::opt_span(dx, n * 2, "ln bwd dx");
  hc::span(gamma, (long long)D * 4, "ln bwd gamma");
  hc::span(mean, (long long)T * 4, "ln bwd mean");
  hc::span(rstd, (long long)T * 4, "ln bwd rstd");
  hc::opt_span(dgamma, (long long)D * 4, "ln bwd dgamma");
  hc::opt_span(dbeta, (long long)D * 4, "ln bwd dbeta");
  hc::opt_span(dbias, (long long)D * 4, "ln bwd dbias");
  const int blocks = std::min(512, (T + 7) / 8);  // the kernel's partial-sum grid (csrc/kernels/norm.hip)
  hc::span(work, (long long)blocks * 3 * D * 4, "ln bwd work");
  hc::span(seed, 4, "ln bwd seed");
  hc::opt_span(row_map, (long long)T * 4, "ln bwd row_map");
  if (nblk_out) *nblk_out = blocks;
  return 0;
}
int fd_emb_fwd(const void*, int, const void*, const void*, const float*, const float*, void*, float*, float*, int, int,
               int, float, const uint32_t*, uint32_t, uint32_t, float, const int*, int* ln_epoch,
               unsigned long long* ln_stats, long long ln_stats_n, long long* sorted, long long* perm, hipStream_t) {
  ++hc::calls;
  hc::opt_span(ln_epoch, 4, "emb ln_epoch");
  hc::opt_span(ln_stats, ln_stats_n * 8, "emb ln_stats");
  if ((sorted == nullptr) != (perm == nullptr)) hc::violations.push_back("emb_fwd: sorted without perm");
  return 0;
}
int fd_emb_bwd(const void* dy, const void*, int, const long long* sorted, const long long* perm, const void*,
               const void*, const float*, const float*, const float*, float* dword, float* dpos, float*, float*,
               float* dz, float* work, int T, int, int, int P, int V, int D, const uint32_t*, uint32_t, uint32_t, float,
               int, unsigned char* now, unsigned char* ever, const int*, const int*, int ncs,
               const float* const* cs_parts, float* const* cs_outs, const int* cs_nblk, const int* cs_stride,
               const int* cs_D, const int* cs_nout, const int*, hipStream_t) {
  ++hc::calls;
  if (ncs < 0 || ncs > 32) hc::violations.push_back("emb_bwd: column-sum job count");
  for (int i = 0; i < ncs; ++i) {
    hc::span(cs_parts[i], (long long)cs_nblk[i] * cs_stride[i] * 4, "emb_bwd colsum part");
    for (int k = 0; k < cs_nout[i]; ++k) hc::opt_span(cs_outs[3 * i + k], (long long)cs_D[i] * 4, "emb_bwd colsum out");
  }
  hc::span(dy, (long long)T * D * 2, "emb_bwd dy");
  hc::span(sorted, (long long)T * 8, "emb_bwd sorted");
  hc::span(perm, (long long)T * 8, "emb_bwd perm");
  hc::span(dz, (long long)T * D * 4, "emb_bwd dz");
  // word-gradient pieces [T][D], then the LayerNorm partials [min(256, ceil(T / 8))][3][D]
  hc::span(work, ((long long)T * D + (long long)std::min(256, (T + 7) / 8) * 3 * D) * 4, "emb_bwd work");
  hc::span(dword, (long long)V * D * 4, "emb_bwd dword");
  hc::span(dpos, (long long)P * D * 4, "emb_bwd dpos");
  hc::opt_span(now, V, "emb_bwd now");
  hc::opt_span(ever, V, "emb_bwd ever");
  return 0;
}
int fd_gather_rows2(const void* a, const void* b, void* oa, void* ob, const long long* idx, int n, int d_bytes,
                    hipStream_t) {
  ++hc::calls;
  hc::span(oa, (long long)n * d_bytes, "gather_rows2 oa");
  hc::span(ob, (long long)n * d_bytes, "gather_rows2 ob");
  hc::span(idx, (long long)n * 8, "gather_rows2 idx");
  (void)a; (void)b;  // rows named by device indices
  return 0;
}
int fd_scatter_rows2(const void* a, const void* b, void* oa, void* ob, const long long* idx, int nsrc, int T,
                     int d_bytes, hipStream_t) {
  ++hc::calls;
  hc::span(a, (long long)nsrc * d_bytes, "scatter_rows2 a");
  hc::span(b, (long long)nsrc * d_bytes, "scatter_rows2 b");
  hc::span(oa, (long long)T * d_bytes, "scatter_rows2 oa");
  hc::span(ob, (long long)T * d_bytes, "scatter_rows2 ob");
  hc::span(idx, (long long)nsrc * 8, "scatter_rows2 idx");
  return 0;
}
int fd_pack(const void* mask, int mask_bytes, const void* ids, int ids_bytes, int B, int S, int rows, int* row_map,
            int* cu, long long* ids_packed, int* step, uint32_t* seed, long long* cls_rows, int* cls_rmap,
            hipStream_t) {
  hc::opt_span(cls_rmap, (long long)B * 4, "pack cls_rmap");
  ++hc::calls;
  hc::opt_span(cls_rows, (long long)B * 8, "pack cls_rows");
  hc::opt_span(step, 4, "pack step");
  hc::opt_span(seed, 4, "pack seed");
  hc::span(mask, (long long)B * S * mask_bytes, "pack mask");
  hc::span(ids, (long long)B * S * ids_bytes, "pack ids");
  hc::span(row_map, (long long)rows * 4, "pack row_map");
  hc::span(cu, (long long)(B + 1) * 4, "pack cu");
  hc::span(ids_packed, (long long)rows * 8, "pack ids_packed");
  return 0;
}
int fd_colsum_bf16(const void*, int, int, float*, float*, int, int, int* nblk_out, hipStream_t) {
  ++hc::calls;
  if (nblk_out) *nblk_out = 1;
  return 0;
}
int fd_colsum_bf16_batched(int n, const void* const* xs, const int* T, const int* N, float* const* parts,
                           hipStream_t) {
  ++hc::calls;
  for (int i = 0; i < n; ++i) {
    hc::span(xs[i], (long long)T[i] * N[i] * 2, "colsum_bf16_batched x");
    hc::span(parts[i], (long long)((T[i] + 31) / 32) * N[i] * 4, "colsum_bf16_batched part");
  }
  return 0;
}
int fd_colsum_batched(int, const float* const*, float* const*, const int*, const int*, const int*, const int*,
                      const int*, hipStream_t) { ++hc::calls; return 0; }
int fd_rank_sort(const void*, int, int, long long*, long long*, hipStream_t) { ++hc::calls; return 0; }
int fd_head_fwd(const void* hidden, int B, int S, int D, const float* W, const float* bias, const uint32_t* seed,
                uint32_t, uint32_t, float, const long long* labels, float* logits, float* loss, float* dlogits,
                float* row_loss, const int* cls, int T, const float* tlogits, float, float, float* loss_acc,
                hipStream_t) {
  ++hc::calls;
  hc::opt_span(loss_acc, 4, "head loss_acc");
  hc::span(hidden, (long long)T * D * 2, "head hidden");
  hc::span(W, 2LL * D * 4, "head W");
  hc::span(bias, 8, "head bias");
  hc::span(logits, 2LL * B * 4, "head logits");
  if (!cls && (long long)B * S > T) hc::violations.push_back("head: padded rows beyond hidden");
  hc::opt_span(cls, (long long)B * 4, "head cls");
  if (labels) {
    hc::span(labels, (long long)B * 8, "head labels");
    hc::span(loss, 4, "head loss");
    hc::span(dlogits, 2LL * B * 4, "head dlogits");
    hc::span(row_loss, (long long)B * 4, "head row_loss");
  }
  hc::opt_span(tlogits, 2LL * B * 4, "head teacher logits");
  hc::span(seed, 4, "head seed");
  return 0;
}
int fd_head_bwd(const void* hidden, int B, int S, int D, const float* W, const uint32_t* seed, uint32_t, uint32_t,
                float, const float* dlogits, float* dW, float* db, void* dhidden, int, const int* cls, int T,
                const float* gscale, const int* own, hipStream_t) {
  ++hc::calls;
  hc::opt_span(own, (B + 1LL) * 4, "head bwd own");
  hc::span(hidden, (long long)T * D * 2, "head bwd hidden");
  hc::span(dhidden, (long long)T * D * 2, "head bwd dhidden");
  hc::span(W, 2LL * D * 4, "head bwd W");
  hc::span(dlogits, 2LL * B * 4, "head bwd dlogits");
  hc::span(dW, 2LL * D * 4, "head bwd dW");
  hc::span(db, 8, "head bwd db");
  hc::opt_span(cls, (long long)B * 4, "head bwd cls");
  hc::opt_span(gscale, 4, "head bwd gscale");
  hc::span(seed, 4, "head bwd seed");
  (void)S;
  return 0;
}
int fd_head_ln_bwd(const void* hidden, int B, int T, int D, const float* W, const float* bias, const uint32_t* seed,
                   uint32_t, uint32_t, float, const long long* labels, float* logits, float* loss, float* dlogits,
                   float* row_loss, float* loss_acc, float* dW, float* db, int, const int* own, const float* tlogits,
                   float, float, const void* z, const float* gamma, const float* mean, const float* rstd, void* dz,
                   void* dx, float* part, uint32_t, uint32_t thr, float, const int* row_map, int* nblk_out,
                   hipStream_t) {
  ++hc::calls;
  const long long td = (long long)T * D;
  if (B > T) hc::violations.push_back("head_ln_bwd: B > T");
  hc::span(hidden, td * 2, "head_ln hidden");
  hc::span(W, 2LL * D * 4, "head_ln W");
  hc::span(bias, 8, "head_ln bias");
  hc::span(labels, (long long)B * 8, "head_ln labels");
  hc::span(logits, 2LL * B * 4, "head_ln logits");
  hc::span(loss, 4, "head_ln loss");
  hc::span(dlogits, 2LL * B * 4, "head_ln dlogits");
  hc::span(row_loss, (long long)B * 4, "head_ln row_loss");
  hc::opt_span(loss_acc, 4, "head_ln loss_acc");
  hc::span(dW, 2LL * D * 4, "head_ln dW");
  hc::span(db, 8, "head_ln db");
  hc::opt_span(own, (B + 1LL) * 4, "head_ln own");
  hc::opt_span(tlogits, 2LL * B * 4, "head_ln teacher logits");
  hc::span(z, td * 2, "head_ln z");
  hc::span(gamma, (long long)D * 4, "head_ln gamma");
  hc::span(mean, (long long)T * 4, "head_ln mean");
  hc::span(rstd, (long long)T * 4, "head_ln rstd");
  hc::span(dz, td * 2, "head_ln dz");
  if (thr) hc::span(dx, td * 2, "head_ln dx");
  const int nlb = (T + 15) / 16;
  hc::span(part, (long long)nlb * 3 * D * 4, "head_ln part");
  hc::opt_span(row_map, (long long)T * 4, "head_ln row_map");
  hc::span(seed, 4, "head_ln seed");
  if (nblk_out) *nblk_out = nlb;
  return 0;
}
int fd_eval_metrics(const float*, const long long*, int, double*, long long*, float*, long long*, hipStream_t) {
  ++hc::calls;
  return 0;
}
int fd_adam(float* p, const float* g, float* m, float* v, void* shadow, long long n, const int* step, float, float,
            float, float, float, int, const unsigned char* touched, const unsigned char* now, long long skip_off,
            long long skip_rows, int row_len, const long long* runs, int nruns, long long run_total4, hipStream_t) {
  ++hc::calls;
  hc::span(p, n * 4, "adam p");
  hc::span(g, n * 4, "adam g");
  hc::span(m, n * 4, "adam m");
  hc::span(v, n * 4, "adam v");
  hc::opt_span(shadow, n * 2, "adam shadow");
  hc::span(step, 4, "adam step");
  if (touched) {
    hc::span(touched, skip_rows, "adam touched");
    hc::opt_span(now, skip_rows, "adam now");
    if (skip_off < 0 || skip_off + skip_rows * row_len > n) hc::violations.push_back("adam: skip range");
  }
  if (runs) {  // the kernel indexes [start4, start4 + count4) of every run (csrc/kernels/head_optim.hip)
    hc::span(runs, (long long)nruns * 3 * 8, "adam runs");
    long long pre = 0;
    for (int i = 0; i < nruns; ++i) {
      const long long s4 = runs[3 * i], c4 = runs[3 * i + 1], p4 = runs[3 * i + 2];
      if (s4 < 0 || c4 <= 0 || (s4 + c4) * 4 > n) hc::violations.push_back("adam: run outside the arena");
      if (p4 != pre) hc::violations.push_back("adam: run prefix");
      pre += c4;
    }
    if (pre != run_total4) hc::violations.push_back("adam: run total");
  }
  return 0;
}
int fd_step(int*, uint32_t*, hipStream_t) { ++hc::calls; return 0; }
int fd_scale_cast(float*, void*, long long, float, hipStream_t) { ++hc::calls; return 0; }
int fd_axpby(float*, const float*, const float*, float, float, long long, hipStream_t) { ++hc::calls; return 0; }
}  // extern "C"

// ------------------------------------------------------------------ driver
namespace {
int failures = 0;

at::Tensor T_(at::IntArrayRef shape, at::ScalarType dt) {
  at::Tensor t = at::zeros(shape, at::TensorOptions().dtype(dt));
  hc::reg(t);
  return t;
}

template <typename F>
void expect_ok(const char* name, F f) {
  const size_t v0 = hc::violations.size();
  const int c0 = hc::calls;
  try {
    f();
  } catch (const c10::Error& e) {
    std::printf("FAIL %s: unexpected rejection: %s\n", name, e.what_without_backtrace());
    ++failures;
    return;
  }
  if (hc::calls == c0) {
    std::printf("FAIL %s: no launcher was called\n", name);
    ++failures;
  }
  for (size_t i = v0; i < hc::violations.size(); ++i) {
    std::printf("FAIL %s: %s\n", name, hc::violations[i].c_str());
    ++failures;
  }
}

template <typename F>
void expect_reject(const char* name, F f) {
  const int c0 = hc::calls;
  bool threw = false;
  try {
    f();
  } catch (const c10::Error&) {
    threw = true;
  }
  if (!threw) {
    std::printf("FAIL %s: accepted a call the kernels do not support\n", name);
    ++failures;
  } else if (hc::calls != c0) {
    std::printf("FAIL %s: rejected only after launching\n", name);
    ++failures;
  }
}

const c10::optional<at::Tensor> none = c10::nullopt;
}  // namespace

int main() {
  const auto bf = at::kBFloat16, f32 = at::kFloat, i32 = at::kInt, i64 = at::kLong;
  // ---- GEMMs: y = x W^T + b (NT), dx = dy W (NN), dW (TN); the DistilBERT shapes at a packed bs32 step
  {
    auto x = T_({2688, 768}, bf), w = T_({2304, 768}, bf), y = T_({2688, 2304}, bf), b = T_({2304}, f32);
    expect_ok("gemm NT bias", [&] { gemm(0, 1, x, w, y, b, none, none, none, false, none); });
    auto w1 = T_({3072, 768}, bf), g = T_({2688, 3072}, bf), u = T_({2688, 3072}, bf), b1 = T_({3072}, f32);
    expect_ok("gemm NT bias+gelu", [&] { gemm(0, 2, x, w1, g, b1, u, none, none, false, none); });
    auto dy = T_({2688, 768}, bf), w2t = T_({3072, 768}, bf), du = T_({2688, 3072}, bf), gout = T_({2688, 3072}, bf);
    expect_ok("gemm NT gelu' + remat", [&] { gemm(0, 3, dy, w2t, du, none, u, none, none, false, gout); });
    auto res = T_({2688, 768}, bf), wt = T_({768, 3072}, bf), dx = T_({2688, 768}, bf);
    expect_ok("gemm NT residual", [&] { gemm(0, 4, du, wt, dx, none, none, res, none, false, none); });
    auto w2 = T_({768, 3072}, bf);
    expect_ok("gemm NN", [&] { gemm(1, 0, dy, w2, du, none, none, none, none, false, none); });
    auto dW = T_({2304, 768}, f32), dq = T_({2688, 2304}, bf), ws = T_({8 * 2304 * 768}, f32);
    expect_ok("gemm TN", [&] { gemm(2, 5, dq, x, dW, none, none, none, ws, false, none); });
    auto cs = T_({21 * 3072}, f32);
    expect_ok("gemm colsum", [&] { gemm_colsum(3, dy, w2t, du, u, none, cs, gout); });
    // rejections
    auto xk = T_({2688, 700}, bf), wk = T_({2304, 700}, bf);
    expect_reject("gemm K % 64", [&] { gemm(0, 1, xk, wk, y, b, none, none, none, false, none); });
    expect_reject("gemm C shape", [&] { gemm(0, 1, x, w, dx, b, none, none, none, false, none); });
    expect_reject("gemm bias size", [&] { gemm(0, 1, x, w, y, b1, none, none, none, false, none); });
    auto xf = T_({2688, 768}, f32);
    expect_reject("gemm dtype", [&] { gemm(0, 1, xf, w, y, b, none, none, none, false, none); });
    // (bias+GELU without u: a forward without autograd keeps only the activation)
    expect_ok("gemm NT bias+gelu, no u", [&] { gemm(0, 2, x, w1, g, b1, none, none, none, false, none); });
    expect_reject("gemm aux missing", [&] { gemm(0, 3, dy, w2t, du, none, none, none, none, false, none); });
    expect_reject("gemm aux shape", [&] { gemm(0, 2, x, w1, g, b1, y, none, none, false, none); });
    expect_reject("gemm aux_out epi", [&] { gemm(0, 1, x, w, y, b, none, none, none, false, gout); });
    auto xt = x.t();
    expect_reject("gemm non-contiguous", [&] { gemm(0, 1, xt, w, y, b, none, none, none, false, none); });
    auto cs_small = T_({3072}, f32);
    expect_reject("gemm colsum size", [&] { gemm_colsum(3, dy, w2t, du, u, none, cs_small, gout); });
    // batched bf16 column-sum partials (per-layer qkv-bias partials at the end of the backward)
    auto p1 = T_({84 * 2304}, f32), p2 = T_({84 * 3072}, f32), p_small = T_({83 * 2304}, f32);
    expect_ok("colsum_bf16_batched", [&] { colsum_bf16_batched({dq, du}, {p1, p2}, {2304, 3072}); });
    expect_reject("colsum_bf16_batched part size", [&] { colsum_bf16_batched({dq}, {p_small}, {2304}); });
    expect_reject("colsum_bf16_batched N", [&] { colsum_bf16_batched({dq}, {p1}, {2303}); });
    expect_reject("colsum_bf16_batched dtype", [&] { colsum_bf16_batched({p1}, {p1}, {2304}); });
  }
  // ---- all-layer weight gradients (with and without the fused Adam epilogue)
  {
    std::vector<at::Tensor> As, Bs, Cs, st;
    const int64_t shapes[4][2] = {{2304, 768}, {768, 768}, {3072, 768}, {768, 3072}};
    for (auto& sh : shapes) {
      As.push_back(T_({2688, sh[0]}, bf));
      Bs.push_back(T_({2688, sh[1]}, bf));
      Cs.push_back(T_({sh[0], sh[1]}, f32));
      st.push_back(T_({sh[0] * sh[1]}, f32));
      st.push_back(T_({sh[0] * sh[1]}, f32));
      st.push_back(T_({sh[0] * sh[1]}, f32));
      st.push_back(T_({sh[0] * sh[1]}, bf));
    }
    st.push_back(T_({1}, i32));
    const std::vector<double> hp = {2e-5, 0.9, 0.999, 1e-8, 0.0, 0.0};
    std::vector<int64_t> acc(4, 0), acc1 = {0, 1, 0, 0};
    expect_ok("dw_batch", [&] { gemm_dw_batch(As, Bs, Cs, acc, {}, {}, -1); });
    expect_ok("dw_batch adam", [&] { gemm_dw_batch(As, Bs, Cs, acc, st, hp, -1); });
    expect_reject("dw_batch adam+accumulate", [&] { gemm_dw_batch(As, Bs, Cs, acc1, st, hp, -1); });
    auto Bbad = Bs;
    Bbad[2] = T_({2000, 768}, bf);
    expect_reject("dw_batch K mismatch", [&] { gemm_dw_batch(As, Bbad, Cs, acc, {}, {}, -1); });
    // per-problem rows (the pruned last block: padded [CLS] rows)
    auto Amix = As, Bmix = Bs;
    Amix[1] = T_({64, As[1].size(1)}, bf);
    Bmix[1] = T_({64, Bs[1].size(1)}, bf);
    expect_ok("dw_batch mixed K", [&] { gemm_dw_batch(Amix, Bmix, Cs, acc, st, hp, -1); });
    auto Bodd = Bmix;
    Bodd[1] = T_({96, Bs[1].size(1)}, bf);
    auto Aodd = Amix;
    Aodd[1] = T_({96, As[1].size(1)}, bf);
    expect_reject("dw_batch K % 64", [&] { gemm_dw_batch(Aodd, Bodd, Cs, acc, {}, {}, -1); });
    auto Cbad = Cs;
    Cbad[1] = T_({768, 3072}, f32);
    expect_reject("dw_batch C shape", [&] { gemm_dw_batch(As, Bs, Cbad, acc, {}, {}, -1); });
    auto stbad = st;
    stbad[5] = T_({100}, f32);
    expect_reject("dw_batch adam state size", [&] { gemm_dw_batch(As, Bs, Cs, acc, stbad, hp, -1); });
    std::vector<at::Tensor> A33(33, As[1]), B33(33, Bs[1]), C33(33, Cs[1]);
    expect_reject("dw_batch > 32 problems", [&] { gemm_dw_batch(A33, B33, C33, std::vector<int64_t>(33, 0), {}, {}, -1); });
    auto A0 = T_({2688, 768}, bf), B0 = T_({2688, 3072}, bf), C0 = T_({768, 3072}, f32);
    auto A1 = T_({2688, 3072}, bf), B1 = T_({2688, 768}, bf), C1 = T_({3072, 768}, f32), wsp = T_({8 * 2 * 2359296}, f32);
    expect_ok("dw2", [&] { gemm_dw2(A0, B0, C0, A1, B1, C1, wsp, false, {}, {}, false); });
  }
  // ---- split-K small-M GEMM + fused epilogues (splitk.hip)
  {
    auto A = T_({64, 3072}, bf), Bt = T_({768, 3072}, bf), C = T_({64, 768}, bf), ws = T_({256 * 64 * 64 + 64 * 768}, f32);
    auto res = T_({64, 768}, bf), g = T_({768}, f32), b = T_({768}, f32), mean = T_({64}, f32), rstd = T_({64}, f32);
    auto z = T_({64, 768}, bf), dx = T_({64, 768}, bf), cp = T_({64 * 3 * 768}, f32), sd = T_({1}, i32);
    const c10::optional<at::Tensor> o_b = b, o_res = res, o_g = g, o_m = mean, o_r = rstd, o_z = z, o_dx = dx, o_cp = cp,
                                    o_sd = sd;
    expect_ok("splitk bf16", [&] { gemm_splitk(0, A, Bt, C, ws, 0, none, none, none, none, none, none, none, none, none,
                                               none, none, none, 1e-12, none, 0, 0, 1.0, none); });
    expect_ok("splitk ln fwd", [&] { gemm_splitk(6, A, Bt, C, ws, 0, o_b, none, none, o_res, none, o_g, o_b, o_m, o_r,
                                                 o_z, none, none, 1e-12, o_sd, 9, 1000, 1.1, none); });
    expect_ok("splitk ln bwd", [&] { gemm_splitk(7, A, Bt, C, ws, 0, none, none, none, o_res, none, o_g, none, o_m, o_r,
                                                 o_z, o_dx, o_cp, 1e-12, o_sd, 9, 1000, 1.1, none); });
    expect_reject("splitk ln bwd colpart", [&] {
      gemm_splitk(7, A, Bt, C, ws, 0, none, none, none, o_res, none, o_g, none, o_m, o_r, o_z, o_dx,
                  c10::optional<at::Tensor>(T_({64 * 768}, f32)), 1e-12, o_sd, 9, 1000, 1.1, none); });
    expect_reject("splitk K mismatch", [&] { gemm_splitk(0, A, T_({768, 768}, bf), C, ws, 0, none, none, none, none,
                                                         none, none, none, none, none, none, none, none, 1e-12, none,
                                                         0, 0, 1.0, none); });
    expect_reject("splitk bias missing", [&] { gemm_splitk(1, A, Bt, C, ws, 0, none, none, none, none, none, none, none,
                                                           none, none, none, none, none, 1e-12, none, 0, 0, 1.0, none); });
  }
  // ---- attention (padded and varlen), S up to 512
  {
    const int64_t B = 4, S = 128, H = 12, rows = B * S;
    auto qkv = T_({rows, 3 * H * 64}, bf), kb = T_({B, S}, f32), ctx = T_({rows, H * 64}, bf);
    auto lse = T_({B, H, S}, f32), seed = T_({1}, i32), dctx = T_({rows, H * 64}, bf), delta = T_({B * H * S}, f32);
    auto dqkv = T_({rows, 3 * H * 64}, bf);
    expect_ok("attn fwd", [&] { attn_fwd(qkv, kb, ctx, lse, B, S, H, seed, 16, 429496730, 1.1, none, none); });
    expect_ok("attn bwd", [&] { attn_bwd(qkv, kb, ctx, lse, dctx, delta, dqkv, B, S, H, seed, 16, 0, 1.0, none, none); });
    auto cu = T_({B + 1}, i32), qv = T_({300, 3 * H * 64}, bf), cv = T_({300, H * 64}, bf);
    expect_ok("attn fwd varlen", [&] { attn_fwd(qv, kb, cv, lse, B, S, H, seed, 16, 0, 1.0, cu, none); });
    const int64_t S5 = 512;
    auto q5 = T_({2 * S5, 3 * H * 64}, bf), k5 = T_({2, S5}, f32), c5 = T_({2 * S5, H * 64}, bf), l5 = T_({2, H, S5}, f32);
    expect_ok("attn fwd S=512", [&] { attn_fwd(q5, k5, c5, l5, 2, S5, H, seed, 16, 0, 1.0, none, none); });
    expect_reject("attn S=576", [&] { attn_fwd(q5, k5, c5, l5, 2, 576, H, seed, 16, 0, 1.0, none, none); });
    expect_reject("attn S % 64", [&] { attn_fwd(qkv, kb, ctx, lse, B, 100, H, seed, 16, 0, 1.0, none, none); });
    expect_reject("attn lse size", [&] { attn_fwd(qkv, kb, ctx, l5, B, S, H, seed, 16, 0, 1.0, none, none); });
    auto cu_bad = T_({B}, i32);
    expect_reject("attn cu size", [&] { attn_fwd(qv, kb, cv, lse, B, S, H, seed, 16, 0, 1.0, cu_bad, none); });
    auto dm = T_({B * H * 256}, i64), dm_bad = T_({B * H * 100}, i64);
    expect_ok("attn fwd + keep bits", [&] { attn_fwd(qkv, kb, ctx, lse, B, S, H, seed, 16, 429496730, 1.1, none, dm); });
    expect_ok("attn bwd + keep bits", [&] { attn_bwd(qkv, kb, ctx, lse, dctx, delta, dqkv, B, S, H, seed, 16, 429496730,
                                                     1.1, none, dm); });
    expect_reject("attn dmask size", [&] { attn_fwd(qkv, kb, ctx, lse, B, S, H, seed, 16, 429496730, 1.1, none, dm_bad); });
    expect_reject("attn dmask S=512", [&] { attn_fwd(q5, k5, c5, l5, 2, S5, H, seed, 16, 0, 1.0, none, dm); });
    expect_reject("attn bwd dqkv size", [&] { attn_bwd(qkv, kb, ctx, lse, dctx, delta, ctx, B, S, H, seed, 16, 0, 1.0, none, none); });
    // fused QKV projection + attention (both modes): flags in the LayerNorm state's tail
    auto x = T_({rows, H * 64}, bf), w = T_({3 * H * 64, H * 64}, bf), bq = T_({3 * H * 64}, f32);
    auto stats = T_({4096}, i64), cnt = T_({2}, i32), err = T_({1}, i32);
    for (int64_t mode : {1, 2}) {
      expect_ok("qkv attn fwd", [&] { gemm_attn_fwd(x, w, bq, qkv, kb, ctx, lse, B, S, H, seed, 16, 429496730, 1.1,
                                                   none, dm, 0, stats, cnt, err, 2, none, none, none, none, mode); });
      auto xv = T_({300, H * 64}, bf);
      expect_ok("qkv attn fwd varlen", [&] { gemm_attn_fwd(xv, w, bq, qv, kb, cv, lse, B, S, H, seed, 16, 0, 1.0, cu,
                                                          none, 0, stats, cnt, err, 2, none, none, none, none, mode); });
    }
    expect_reject("qkv attn S=256", [&] { gemm_attn_fwd(x, w, bq, qkv, kb, ctx, lse, 2, 256, H, seed, 16, 0, 1.0, none,
                                                        none, 0, stats, cnt, err, 2, none, none, none, none, 1); });
    expect_reject("qkv attn w shape", [&] { gemm_attn_fwd(x, T_({2 * H * 64, H * 64}, bf), bq, qkv, kb, ctx, lse, B, S, H,
                                                          seed, 16, 0, 1.0, none, none, 0, stats, cnt, err, 2, none,
                                                          none, none, none, 1); });
    expect_reject("qkv attn stats", [&] { gemm_attn_fwd(x, w, bq, qkv, kb, ctx, lse, B, S, H, seed, 16, 0, 1.0, none,
                                                        none, 0, T_({1000}, i64), cnt, err, 2, none, none, none, none,
                                                        1); });
    expect_reject("qkv attn xsite", [&] { gemm_attn_fwd(x, w, bq, qkv, kb, ctx, lse, B, S, H, seed, 16, 0, 1.0, none,
                                                        none, 0, stats, cnt, err, 127, none, none, none, none, 1); });
    expect_ok("attn bwd proj", [&] { attn_bwd_proj(qkv, kb, ctx, lse, x, T_({H * 64, H * 64}, bf), dqkv, B, S, H, seed, 16,
                                                  429496730, 1.1, none, dm); });
    expect_ok("attn bwd proj varlen", [&] { attn_bwd_proj(qv, kb, cv, lse, T_({300, H * 64}, bf), T_({H * 64, H * 64}, bf),
                                                         T_({300, 3 * H * 64}, bf), B, S, H, seed, 16, 0, 1.0, cu, none); });
    expect_reject("attn bwd proj S=256", [&] { attn_bwd_proj(qkv, kb, ctx, lse, x, T_({H * 64, H * 64}, bf), dqkv, 2, 256,
                                                            H, seed, 16, 0, 1.0, none, none); });
    expect_reject("attn bwd proj w shape", [&] { attn_bwd_proj(qkv, kb, ctx, lse, x, T_({H * 64, 64}, bf), dqkv, B, S, H,
                                                              seed, 16, 0, 1.0, none, none); });
    expect_reject("qkv attn mode", [&] { gemm_attn_fwd(x, w, bq, qkv, kb, ctx, lse, B, S, H, seed, 16, 0, 1.0, none,
                                                       none, 0, stats, cnt, err, 2, none, none, none, none, 3); });
  }
  // ---- LayerNorm fwd / bwd
  {
    const int64_t Tn = 2688, D = 768;
    auto x = T_({Tn, D}, bf), r = T_({Tn, D}, bf), ga = T_({D}, f32), be = T_({D}, f32), y = T_({Tn, D}, bf);
    auto mean = T_({Tn}, f32), rstd = T_({Tn}, f32), seed = T_({1}, i32), rm = T_({Tn}, i32);
    expect_ok("ln fwd", [&] { ln_fwd(x, r, ga, be, y, mean, rstd, 1e-12, seed, 17, 429496730, 1.1, rm); });
    auto dz = T_({Tn, D}, bf), dx = T_({Tn, D}, bf), dg = T_({D}, f32), db = T_({D}, f32), dbias = T_({D}, f32);
    auto work = T_({336 * 3 * D}, f32);
    expect_ok("ln bwd", [&] { ln_bwd(x, x, r, ga, mean, rstd, dz, dx, dg, db, dbias, work, seed, 17, 429496730, 1.1,
                                     false, rm, true, false); });
    auto small = T_({100 * 3 * D}, f32);
    expect_reject("ln bwd work", [&] { ln_bwd(x, x, r, ga, mean, rstd, dz, dx, dg, db, dbias, small, seed, 17, 0, 1.0,
                                              false, none, false, false); });
    expect_reject("ln bwd dx with dropout", [&] { ln_bwd(x, x, r, ga, mean, rstd, dz, none, dg, db, dbias, work, seed,
                                                         17, 429496730, 1.1, false, none, false, false); });
    expect_ok("ln bwd from z", [&] { ln_bwd(x, x, none, ga, mean, rstd, dz, dx, dg, db, dbias, work, seed, 17, 429496730,
                                            1.1, false, rm, true, true); });
    expect_reject("ln bwd z + residual", [&] { ln_bwd(x, x, r, ga, mean, rstd, dz, dx, dg, db, dbias, work, seed, 17, 0,
                                                      1.0, false, none, false, true); });
    auto g2 = T_({1024}, f32);
    expect_reject("ln fwd D", [&] { ln_fwd(x, r, g2, g2, y, mean, rstd, 1e-12, seed, 17, 0, 1.0, none); });
    auto rm_bad = T_({10}, i32);
    expect_reject("ln fwd row_map", [&] { ln_fwd(x, r, ga, be, y, mean, rstd, 1e-12, seed, 17, 0, 1.0, rm_bad); });
    // LayerNorm fused into the N = 768 GEMM (forward: out_lin / lin2; backward: the dX GEMM)
    auto a = T_({Tn, 3072}, bf), wt = T_({D, 3072}, bf), bias = T_({D}, f32), z = T_({Tn, D}, bf);
    auto stats = T_({2 * (Tn + 128) * (D / 64)}, i64), cnt = T_({2}, i32), err = T_({1}, i32);
    auto cp = T_({((Tn + 63) / 64) * 3 * D}, f32);
    expect_ok("gemm_ln fwd", [&] { gemm_ln(false, a, wt, y, bias, r, ga, be, mean, rstd, z, none, none, stats, cnt, err,
                                           1e-12, seed, 17, 429496730, 1.1, rm, -1, 0); });
    expect_ok("gemm_ln bwd", [&] { gemm_ln(true, a, wt, dz, none, r, ga, none, mean, rstd, z, dx, cp, stats, cnt, err,
                                           1e-12, seed, 17, 429496730, 1.1, rm, -1, 0); });
    expect_reject("gemm_ln bwd without z", [&] { gemm_ln(true, a, wt, dz, none, r, ga, none, mean, rstd, none, dx, cp,
                                                         stats, cnt, err, 1e-12, seed, 17, 0, 1.0, none, -1, 0); });
    expect_reject("gemm_ln bwd dropout without dx", [&] {
      gemm_ln(true, a, wt, dz, none, r, ga, none, mean, rstd, z, none, cp, stats, cnt, err, 1e-12, seed, 17, 429496730,
              1.1, rm, -1, 0); });
    auto stats_small = T_({100}, i64);
    expect_reject("gemm_ln stats size", [&] { gemm_ln(false, a, wt, y, bias, r, ga, be, mean, rstd, z, none, none,
                                                      stats_small, cnt, err, 1e-12, seed, 17, 0, 1.0, none, -1, 0); });
    expect_reject("gemm_ln fwd without beta", [&] { gemm_ln(false, a, wt, y, bias, r, ga, none, mean, rstd, z, none,
                                                            none, stats, cnt, err, 1e-12, seed, 17, 0, 1.0, none, -1, 0); });
    expect_reject("gemm_ln xsite range", [&] { gemm_ln(false, a, wt, y, bias, r, ga, be, mean, rstd, z, none, none,
                                                       stats, cnt, err, 1e-12, seed, 17, 0, 1.0, none, -1, 128); });
    auto cp_small = T_({3 * D}, f32);
    expect_reject("gemm_ln colpart size", [&] { gemm_ln(true, a, wt, dz, none, r, ga, none, mean, rstd, z, dx, cp_small,
                                                        stats, cnt, err, 1e-12, seed, 17, 0, 1.0, none, -1, 0); });
  }
  // ---- head (+ fused distillation loss)
  {
    const int64_t B = 32, S = 128, D = 768;
    auto hid = T_({B * S, D}, bf), W = T_({2, D}, f32), bias = T_({2}, f32), seed = T_({1}, i32);
    auto lab = T_({B}, i64), logits = T_({B, 2}, f32), loss = T_({}, f32), dlog = T_({B, 2}, f32), rl = T_({B}, f32);
    auto tl = T_({B, 2}, f32);
    expect_ok("head fwd", [&] { head_fwd(hid, B, S, W, bias, seed, 2, 0, 1.0, lab, logits, loss, dlog, rl, none,
                                         none, 1.0, 1.0, none); });
    const c10::optional<at::Tensor> lacc = T_({1}, f32);
    expect_ok("head fwd loss_acc", [&] { head_fwd(hid, B, S, W, bias, seed, 2, 0, 1.0, lab, logits, loss, dlog, rl,
                                                  none, none, 1.0, 1.0, lacc); });
    expect_ok("head fwd kd", [&] { head_fwd(hid, B, S, W, bias, seed, 2, 0, 1.0, lab, logits, loss, dlog, rl, none, tl,
                                            2.0, 0.5, none); });
    expect_reject("head kd without labels", [&] { head_fwd(hid, B, S, W, bias, seed, 2, 0, 1.0, none, logits, none,
                                                           none, none, none, tl, 2.0, 0.5, none); });
    expect_reject("head kd T <= 0", [&] { head_fwd(hid, B, S, W, bias, seed, 2, 0, 1.0, lab, logits, loss, dlog, rl,
                                                   none, tl, 0.0, 0.5, none); });
    auto dW = T_({2, D}, f32), db = T_({2}, f32), dh = T_({B * S, D}, bf);
    expect_ok("head bwd", [&] { head_bwd(hid, B, S, W, seed, 2, 0, 1.0, dlog, dW, db, dh, false, none, none, none); });
    auto hid_small = T_({B * S - 1, D}, bf);
    expect_reject("head bwd hidden size", [&] { head_bwd(hid_small, B, S, W, seed, 2, 0, 1.0, dlog, dW, db, hid_small,
                                                         false, none, none, none); });
  }
  // ---- Adam over an arena with a run table (the fused-step remainder)
  {
    const int64_t n = 4096;
    auto p = T_({n}, f32), g = T_({n}, f32), m = T_({n}, f32), v = T_({n}, f32), sh = T_({n}, bf), step = T_({1}, i32);
    auto runs = T_({2, 3}, i64);
    auto rp = runs.data_ptr<int64_t>();
    rp[0] = 0; rp[1] = 64; rp[2] = 0; rp[3] = 512; rp[4] = 256; rp[5] = 64;
    expect_ok("adam runs", [&] { adam(p, g, m, v, sh, step, 2e-5, 0.9, 0.999, 1e-8, 0, false, none, none, 0, 0, 4,
                                      runs, 320, 768); });
    expect_reject("adam run end outside", [&] { adam(p, g, m, v, sh, step, 2e-5, 0.9, 0.999, 1e-8, 0, false, none,
                                                     none, 0, 0, 4, runs, 320, 4096); });
    auto g_small = T_({n - 4}, f32);
    expect_reject("adam sizes", [&] { adam(p, g_small, m, v, sh, step, 2e-5, 0.9, 0.999, 1e-8, 0, false, none, none,
                                           0, 0, 4, none, 0, 0); });
    // the sparse word-embedding rows (64 rows of 64)
    auto ever = T_({64}, at::kByte), now = T_({64}, at::kByte), ever_small = T_({10}, at::kByte);
    expect_ok("adam rows", [&] { adam_rows(p, g, m, v, sh, step, 2e-5, 0.9, 0.999, 1e-8, ever, now, 64); });
    expect_reject("adam rows flags", [&] { adam_rows(p, g, m, v, sh, step, 2e-5, 0.9, 0.999, 1e-8, ever_small, now,
                                                     64); });
    expect_reject("adam rows row_len", [&] { adam_rows(p, g, m, v, sh, step, 2e-5, 0.9, 0.999, 1e-8, ever, now, 6); });
  }
  // ---- embedding backward (work = pieces + LayerNorm partials)
  {
    const int64_t Tn = 2688, D = 768, V = 1000, P = 512;
    auto dy = T_({Tn, D}, bf), ids = T_({Tn}, i64), srt = T_({Tn}, i64), prm = T_({Tn}, i64);
    auto word = T_({V, D}, bf), pos = T_({P, D}, bf), ga = T_({D}, f32), mean = T_({Tn}, f32), rstd = T_({Tn}, f32);
    auto dword = T_({V, D}, f32), dpos = T_({P, D}, f32), dg = T_({D}, f32), db = T_({D}, f32), dz = T_({Tn, D}, f32);
    auto work = T_({Tn * D + 256 * 3 * D}, f32), work_small = T_({Tn * D}, f32), seed = T_({1}, i32);
    expect_ok("emb bwd", [&] { emb_bwd(dy, ids, srt, prm, word, pos, ga, mean, rstd, dword, dpos, dg, db, dz, work,
                                       128, seed, 1, 0, 1.0, false, none, none, none, none); });
    expect_reject("emb bwd work", [&] { emb_bwd(dy, ids, srt, prm, word, pos, ga, mean, rstd, dword, dpos, dg, db, dz,
                                                work_small, 128, seed, 1, 0, 1.0, false, none, none, none, none); });
    // the backward's deferred column sums riding on the tail launch
    auto part = T_({21 * 3 * D}, f32), part_small = T_({20 * 3 * D}, f32);
    std::vector<std::vector<c10::optional<at::Tensor>>> outs = {{dg, db, c10::optional<at::Tensor>(T_({D}, f32))}};
    expect_ok("emb bwd + colsum jobs", [&] { emb_bwd(dy, ids, srt, prm, word, pos, ga, mean, rstd, dword, dpos, dg, db,
                                                     dz, work, 128, seed, 1, 0, 1.0, false, none, none, none, none,
                                                     {part}, outs, {21}, {3 * D}, {D}, {0}); });
    expect_reject("emb bwd colsum part", [&] { emb_bwd(dy, ids, srt, prm, word, pos, ga, mean, rstd, dword, dpos, dg,
                                                       db, dz, work, 128, seed, 1, 0, 1.0, false, none, none, none,
                                                       none, {part_small}, outs, {21}, {3 * D}, {D}, {0}); });
  }
  // ---- unpadded layout
  {
    auto mask = T_({32, 128}, i64), ids = T_({32, 128}, i64), rm = T_({2688}, i32), cu = T_({33}, i32);
    auto ip = T_({2688}, i64);
    expect_ok("pack", [&] { pack(mask, ids, rm, cu, ip, none, none, none, none); });
    {
      auto ga = T_({300, 768}, bf), gb = T_({300, 768}, bf), go = T_({64, 768}, bf), go2 = T_({64, 768}, bf);
      auto gi = T_({64}, i64);
      expect_ok("gather_rows2", [&] { gather_rows2(ga, gb, go, go2, gi); });
      expect_ok("scatter_rows2", [&] { scatter_rows2(go, go2, ga, gb, gi, 32); });
      auto gbad = T_({63, 768}, bf);
      expect_reject("gather_rows2 shapes", [&] { gather_rows2(ga, gb, gbad, go2, gi); });
      expect_reject("scatter_rows2 nsrc", [&] { scatter_rows2(go, go2, ga, gb, gi, 65); });
    }
    auto st1 = T_({1}, i32);
    expect_ok("pack + counters", [&] { pack(mask, ids, rm, cu, ip, st1, st1, none, none); });
    auto stf = T_({1}, f32);
    expect_reject("pack counter dtype", [&] { pack(mask, ids, rm, cu, ip, stf, none, none, none); });
    auto cu_bad = T_({32}, i32);
    expect_reject("pack cu", [&] { pack(mask, ids, rm, cu_bad, ip, none, none, none, none); });
  }
  if (failures) {
    std::printf("binding host check: %d failure(s)\n", failures);
    return 1;
  }
  std::printf("binding host check: ok (%d launcher calls validated)\n", hc::calls);
  return 0;
}
