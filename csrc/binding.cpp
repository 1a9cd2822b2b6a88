// PyTorch binding of the gfx950 kernel library (csrc/kernels/*.hip).
//
// Every entry point validates device, dtype, contiguity and the shapes the
// kernel's grid assumes BEFORE launching (a mis-shaped launch of a hand-written
// kernel can fault the GPU), then launches on the caller's current HIP stream so
// the ops are stream-ordered and capturable into HIP graphs.
#ifdef FD_HOST_VALIDATION
// Host-only build of this validation layer (csrc/host_check/, tests/test_host_sanitizers.py):
// compiled with g++ and ASan/UBSan against CPU ATen, launchers replaced by stubs that check
// every extent the kernels would touch against the buffers the test registered.  Only the
// device-placement check and the stream query differ; every shape/dtype rule is the same code.
#include <ATen/ATen.h>
typedef struct ihipStream_t* hipStream_t;
namespace py { struct gil_scoped_release {}; }  // (no Python in the host-only build)
#else
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#endif

#include <cstdint>
#include <vector>

#include "kernels/adam_epi.h"

extern "C" {
int fd_gemm(int kind, int epi, const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
            int ldc, const float* bias, void* aux, int ldaux, const void* res, int ldres, float* workspace,
            long long workspace_elems, int accumulate, const FdAdamEpi* adam,
            float* colsum, int* colsum_blocks, hipStream_t st);
int fd_gemm_ex(int kind, int epi, const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
               int ldc, const float* bias, void* aux, int ldaux, const void* res, int ldres, float* workspace,
               long long workspace_elems, int accumulate, const FdAdamEpi* adam,
               float* colsum, int* colsum_blocks, void* aux_out, hipStream_t st);
int fd_gemm_set_cfg(int kind, int cfg, int splits);
int fd_gemm_pf(const void* pf, long long bytes);
int fd_gemm_stamps(unsigned long long* host, int nblocks);
int fd_attn_stamps(unsigned long long* host, int nblocks);
int fd_attn_set_split(int on);
int fd_gemm_dw2(const void* A0, const void* B0, float* C0, int M0, int N0, const void* A1, const void* B1, float* C1,
                int M1, int N1, int K, float* workspace, long long workspace_elems, int accumulate,
                const FdAdamEpi* adams, int defer, int* splits_out, hipStream_t st);
int fd_gemm_dw2_splits(int M0, int N0, int M1, int N1, int K);
int fd_gemm_dw_batch(int n, const FdDwProb* probs, int K, const int* step, const float* hyper, int cfg,
                     const FdAdamRest* rest, hipStream_t st);
int fd_gemm_ln_set_diag(int diag);
int fd_gemm_dwb_set_mix(int mode);
long long fd_gemm_dwb_mixed_launches();
int fd_gemm_splitk(int epi, const void* A, const void* Bt, int M, int N, int K, float* workspace,
                   long long workspace_elems, int splits, const float* bias, void* C, void* aux, void* aux_out,
                   const void* res, float* colsum, int* colsum_blocks, const FdLnEpi* ln, const FdSkHead* hd,
                   int b_mn, hipStream_t st);
int fd_gemm_ln(int bwd, const void* A, const void* Bt, void* C, int M, int N, int K, const float* bias,
               const void* res, int ldres, const FdLnEpi* ln, int cfg, int b_mn, hipStream_t st);
int fd_splitk_reduce_batched(int n, const float* const* slabs, float* const* outs, const long long* numel,
                             const int* splits, const int* accumulate, hipStream_t st);

const char* fd_comm_last_error();
int fd_comm_load(const char* path);
int fd_comm_unique_id_bytes();
int fd_comm_get_unique_id(void* out);
int fd_comm_init(void** comm, int nranks, int rank, const void* id_bytes);
int fd_comm_destroy(void* comm);
int fd_comm_async_error(void* comm);
int fd_comm_wait(void* comm, hipStream_t st, long long timeout_ms);
int fd_comm_abort(void* comm);
int fd_comm_allreduce(void* comm, const void* send, void* recv, long long count, int dtype, int op, hipStream_t st);
int fd_comm_broadcast(void* comm, void* buf, long long count, int dtype, int root, hipStream_t st);
int fd_comm_allgather(void* comm, const void* send, void* recv, long long count, int dtype, hipStream_t st);
int fd_gemm_attn_fwd(const void* x, const void* w, const float* bias, void* qkv, int M, int K, const float* kbias,
                     void* ctx, float* lse, int B, int S, int H, const uint32_t* seed_ptr, uint32_t site, uint32_t thr,
                     float drop_scale, const int* cu, int rows, uint64_t* dmask, int q_live, void* cxc, void* xc,
                     const void* xres, int Bp, uint64_t* flags, int nflags, const int* cnt, int xsite, int* err,
                     int mode, int split, hipStream_t st);
int fd_attn_bwd_proj(const void* qkv, const float* kbias, const void* ctx, const float* lse, const void* dy,
                     const void* w, int M, int K, int splits, void* dqkv, int B, int S, int H,
                     const uint32_t* seed_ptr, uint32_t site, uint32_t thr, float drop_scale, const int* cu, int rows,
                     const uint64_t* dmask, const void* dresc, void* dres, int split, hipStream_t st);
int fd_attn_fwd(const void* qkv, const float* kbias, void* ctx, float* lse, int B, int S, int H,
                const uint32_t* seed_ptr, uint32_t site, uint32_t thr, float drop_scale, const int* cu,
                int rows, uint64_t* dmask, int q_live, void* cxc, void* xc, const void* xres, int Bp,
                int split, hipStream_t st);
int fd_attn_bwd(const void* qkv, const float* kbias, const void* ctx, const float* lse, const void* dctx,
                float* delta, void* dqkv, int B, int S, int H, const uint32_t* seed_ptr, uint32_t site,
                uint32_t thr, float drop_scale, const int* cu, int rows, const uint64_t* dmask, int q_live,
                const void* dresc, void* dres, int split, hipStream_t st);
int fd_mask_to_bias(const void* mask, int mask_bytes, float* bias, long n, hipStream_t st);
int fd_ln_fwd(const void* x, const void* r, const float* gamma, const float* beta, void* y, float* mean,
              float* rstd, int T, int D, float eps, const uint32_t* seed_ptr, uint32_t site, uint32_t thr,
              float dscale, const int* row_map, hipStream_t st);
int fd_ln_bwd(const void* dy, const void* x, const void* r, const float* gamma, const float* mean,
              const float* rstd, void* dz, void* dx, float* dgamma, float* dbeta, float* dbias, float* work, int T,
              int D, const uint32_t* seed_ptr, uint32_t site, uint32_t thr, float dscale, int accumulate,
              const int* row_map, int defer, int* nblk_out, int zin, hipStream_t st);
int fd_emb_fwd(const void* ids, int ids64, const void* word, const void* pos, const float* gamma,
               const float* beta, void* y, float* mean, float* rstd, int T, int S, int D, float eps,
               const uint32_t* seed_ptr, uint32_t site, uint32_t thr, float dscale, const int* row_map, int* ln_epoch,
               unsigned long long* ln_stats, long long ln_stats_n, long long* sorted, long long* perm, hipStream_t st);
int fd_emb_bwd(const void* dy, const void* ids, int ids64, const long long* sorted, const long long* perm,
               const void* word, const void* pos, const float* gamma, const float* mean, const float* rstd,
               float* dword, float* dpos, float* dgamma, float* dbeta, float* dz_buf, float* work, int T, int S,
               int B, int P, int V, int D, const uint32_t* seed_ptr, uint32_t site, uint32_t thr, float dscale,
               int accumulate, unsigned char* now, unsigned char* ever, const int* row_map, const int* cu, int ncs, const float* const* cs_parts, float* const* cs_outs, const int* cs_nblk,
               const int* cs_stride, const int* cs_D, const int* cs_nout, const int* cs_acc, hipStream_t st);
int fd_gather_rows2(const void* a, const void* b, void* oa, void* ob, const long long* idx, int n, int d_bytes,
                    hipStream_t st);
int fd_scatter_rows2(const void* a, const void* b, void* oa, void* ob, const long long* idx, int nsrc, int T,
                     int d_bytes, hipStream_t st);
int fd_pack(const void* mask, int mask_bytes, const void* ids, int ids_bytes, int B, int S, int rows, int* row_map,
            int* cu, long long* ids_packed, int* step, uint32_t* seed, long long* cls_rows, int* cls_rmap,
            hipStream_t st);
int fd_colsum_bf16_batched(int n, const void* const* xs, const int* T, const int* N, float* const* parts,
                           hipStream_t st);
int fd_colsum_bf16(const void* x, int T, int N, float* out, float* work, int accumulate, int defer, int* nblk_out,
                   hipStream_t st);
int fd_colsum_batched(int n, const float* const* parts, float* const* outs, const int* nblk, const int* stride,
                      const int* D, const int* nout, const int* accumulate, hipStream_t st);
int fd_rank_sort(const void* ids, int ids64, int T, long long* sorted, long long* perm, hipStream_t st);
int fd_head_fwd(const void* hidden, int B, int S, int D, const float* W, const float* bias,
                const uint32_t* seed_ptr, uint32_t site, uint32_t thr, float dscale, const long long* labels,
                float* logits, float* loss, float* dlogits, float* row_loss, const int* cls, int T,
                const float* tlogits, float kd_T, float kd_alpha, float* loss_acc, hipStream_t st);
int fd_head_bwd(const void* hidden, int B, int S, int D, const float* W, const uint32_t* seed_ptr, uint32_t site,
                uint32_t thr, float dscale, const float* dlogits, float* dW, float* db, void* dhidden,
                int accumulate, const int* cls, int T, const float* gscale, const int* own, hipStream_t st);
int fd_head_ln_bwd(const void* hidden, int B, int T, int D, const float* W, const float* bias,
                   const uint32_t* seed_ptr, uint32_t hsite, uint32_t hthr, float hdscale, const long long* labels,
                   float* logits, float* loss, float* dlogits, float* row_loss, float* loss_acc, float* dW, float* db,
                   int accumulate, const int* own, const float* tlogits, float kd_T, float kd_alpha, const void* z,
                   const float* gamma, const float* mean, const float* rstd, void* dz, void* dx, float* part,
                   uint32_t site, uint32_t thr, float dscale, const int* row_map, int* nblk_out, hipStream_t st);
int fd_eval_metrics(const float* logits, const long long* labels, int B, double* acc, long long* counts,
                    float* prob1, long long* preds, hipStream_t st);
int fd_adam(float* p, const float* g, float* m, float* v, void* shadow, long long n, const int* step, float lr,
            float b1, float b2, float eps, float wd, int decoupled, const unsigned char* touched,
            const unsigned char* now, long long skip_off, long long skip_rows, int row_len, const long long* runs,
            int nruns, long long run_total4, hipStream_t st);
int fd_adam_rows(float* p, const float* g, float* m, float* v, void* shadow, int rows, int row_len, const int* step,
                 float lr, float b1, float b2, float eps, const unsigned char* ever, const unsigned char* now,
                 hipStream_t st);
int fd_step(int* step, uint32_t* seed, hipStream_t st);
int fd_scale_cast(float* p, void* shadow, long long n, float scale, hipStream_t st);
int fd_axpby(float* dst, const float* x, const float* y, float a, float b, long long n, hipStream_t st);
}

namespace {

#ifdef FD_HOST_VALIDATION
hipStream_t stream() { return nullptr; }
bool on_device(const at::Tensor&) { return true; }  // CPU tensors stand in for device buffers
#else
hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }
bool on_device(const at::Tensor& t) { return t.is_cuda(); }
#endif

void check_rc(int rc, const char* what) { TORCH_CHECK(rc == 0, what, ": kernel launcher rejected arguments (rc=", rc, ")"); }

void need(const at::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(on_device(t), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void need_opt(const c10::optional<at::Tensor>& t, at::ScalarType dt, const char* name) {
  if (t.has_value() && t->defined()) need(*t, dt, name);
}
template <typename T>
T* ptr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}
const uint32_t* seedp(const at::Tensor& s) {
  TORCH_CHECK(on_device(s) && s.scalar_type() == at::kInt && s.numel() >= 1, "seed must be a GPU int32 tensor");
  return reinterpret_cast<const uint32_t*>(s.data_ptr());
}

// Arm the next-launch weight prefetch of the fd_gemm_ex call that follows (same host thread).
void set_prefetch(const c10::optional<at::Tensor>& prefetch, const at::Tensor& like) {
  if (prefetch.has_value() && prefetch->defined() && prefetch->numel() > 0) {
    TORCH_CHECK(prefetch->device() == like.device() && prefetch->is_contiguous(),
                "prefetch must be a contiguous tensor on the GEMM's device");
    fd_gemm_pf(prefetch->data_ptr(), (long long)(prefetch->numel() * prefetch->element_size()));
  } else {
    fd_gemm_pf(nullptr, 0);
  }
}

// kind 0: C[M,N] = A[M,K] B[N,K]^T ; kind 1: C[M,N] = A[M,K] B[K,N] ; kind 2: C[M,N] fp32 = A[K,M]^T B[K,N]
void gemm(int64_t kind, int64_t epi, const at::Tensor& A, const at::Tensor& B, const at::Tensor& C,
          const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& aux,
          const c10::optional<at::Tensor>& res, const c10::optional<at::Tensor>& workspace, bool accumulate,
          const c10::optional<at::Tensor>& aux_out, const c10::optional<at::Tensor>& prefetch = c10::nullopt) {
  // prefetch: the NEXT launch's weight, touched by this GEMM's epilogue (fd_gemm_pf)
  need(A, at::kBFloat16, "A");
  need(B, at::kBFloat16, "B");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm operands must be 2-D");
  int64_t M, N, K;
  if (kind == 0) { M = A.size(0); K = A.size(1); N = B.size(0); TORCH_CHECK(B.size(1) == K, "NT: K mismatch"); }
  else if (kind == 1) { M = A.size(0); K = A.size(1); N = B.size(1); TORCH_CHECK(B.size(0) == K, "NN: K mismatch"); }
  else if (kind == 2) { K = A.size(0); M = A.size(1); N = B.size(1); TORCH_CHECK(B.size(0) == K, "TN: K mismatch"); }
  else TORCH_CHECK(false, "bad gemm kind");
  TORCH_CHECK(C.size(0) == M && C.size(1) == N, "C shape mismatch: got ", C.sizes(), " want [", M, ",", N, "]");
  TORCH_CHECK(K % 64 == 0, "gemm: K must be a multiple of 64, got ", K);
  TORCH_CHECK(N % 64 == 0, "gemm: N must be a multiple of 64, got ", N);
  if (kind == 2) {
    need(C, at::kFloat, "C");
    TORCH_CHECK(M % 128 == 0, "TN gemm: M must be a multiple of 128");
  } else {
    need(C, at::kBFloat16, "C");
  }
  need_opt(bias, at::kFloat, "bias");
  need_opt(aux, at::kBFloat16, "aux");
  need_opt(res, at::kBFloat16, "res");
  need_opt(workspace, at::kFloat, "workspace");
  if (epi == 1 || epi == 2) TORCH_CHECK(bias.has_value() && bias->numel() == N, "bias of size N required");
  // (epi 2: aux = u out, optional -- a forward without autograd keeps only gelu(u))
  if (epi == 3 || (epi == 2 && aux.has_value() && aux->defined()))
    TORCH_CHECK(aux.has_value() && aux->size(0) == M && aux->size(1) == N, "aux [M,N] required");
  if (epi == 4) TORCH_CHECK(res.has_value() && res->size(0) == M && res->size(1) == N, "res [M,N] required");
  need_opt(aux_out, at::kBFloat16, "aux_out");
  if (aux_out.has_value() && aux_out->defined())
    TORCH_CHECK(epi == 3 && kind != 2 && aux_out->size(0) == M && aux_out->size(1) == N,
                "aux_out [M,N] only with the GELU' epilogue");
  const long long ws = (workspace.has_value() && workspace->defined()) ? workspace->numel() : 0;
  set_prefetch(prefetch, A);
  check_rc(fd_gemm_ex((int)kind, (int)epi, A.data_ptr(), B.data_ptr(), C.data_ptr(), (int)M, (int)N, (int)K,
                      (int)A.size(1), (int)B.size(1), (int)N, ptr<float>(bias), ptr<void>(aux), (int)N,
                      ptr<void>(res), (int)N, ptr<float>(workspace), ws, accumulate ? 1 : 0, nullptr, nullptr,
                      nullptr, ptr<void>(aux_out), stream()),
           "gemm");
}

// NT dX GEMM (GELU' or residual epilogue) that also leaves per-M-tile column sums of its bf16
// output in `colsum` ([ceil(M / 128)][N] fp32; returns the tile count) for a deferred
// producer-bias gradient.
// kind 0: B = W^T [N][K] (NT, K-major B); kind 1: B = W [K][N] (NN: the MN-major B through the
// LDS-DMA ring with transposing fragment reads).  Returns 0 tiles (no partials left) only for a
// tile configuration without the fused column-sum epilogue.
int64_t gemm_colsum(int64_t epi, const at::Tensor& A, const at::Tensor& B, const at::Tensor& C,
                    const c10::optional<at::Tensor>& aux, const c10::optional<at::Tensor>& res,
                    const at::Tensor& colsum, const c10::optional<at::Tensor>& aux_out, int64_t kind = 0,
                    const c10::optional<at::Tensor>& prefetch = c10::nullopt) {
  need(A, at::kBFloat16, "A");
  need(B, at::kBFloat16, "B");
  need(C, at::kBFloat16, "C");
  need(colsum, at::kFloat, "colsum");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm_colsum operands must be 2-D");
  TORCH_CHECK(kind == 0 || kind == 1, "gemm_colsum: kind 0 (NT) or 1 (NN)");
  const int64_t M = A.size(0), K = A.size(1), N = kind == 0 ? B.size(0) : B.size(1);
  TORCH_CHECK((kind == 0 ? B.size(1) : B.size(0)) == K && C.size(0) == M && C.size(1) == N,
              "gemm_colsum: shape mismatch");
  TORCH_CHECK(K % 64 == 0 && N % 64 == 0, "gemm_colsum: K % 64 and N % 64 required");
  TORCH_CHECK(epi == 3 || epi == 4, "gemm_colsum: GELU' (3) or residual (4) epilogue");
  need_opt(aux, at::kBFloat16, "aux");
  need_opt(res, at::kBFloat16, "res");
  if (epi == 3) TORCH_CHECK(aux.has_value() && aux->size(0) == M && aux->size(1) == N, "aux [M,N] required");
  if (epi == 4) TORCH_CHECK(res.has_value() && res->size(0) == M && res->size(1) == N, "res [M,N] required");
  TORCH_CHECK(colsum.numel() >= ((M + 127) / 128) * N, "gemm_colsum: colsum needs ceil(M/128) x N floats");
  need_opt(aux_out, at::kBFloat16, "aux_out");
  if (aux_out.has_value() && aux_out->defined())
    TORCH_CHECK(epi == 3 && aux_out->size(0) == M && aux_out->size(1) == N, "aux_out [M,N] only with GELU'");
  int blocks = 0;
  set_prefetch(prefetch, A);
  check_rc(fd_gemm_ex((int)kind, (int)epi, A.data_ptr(), B.data_ptr(), C.data_ptr(), (int)M, (int)N, (int)K,
                      (int)K, (int)B.size(1), (int)N, nullptr, ptr<void>(aux), (int)N, ptr<void>(res), (int)N,
                      nullptr, 0, 0, nullptr, colsum.data_ptr<float>(), &blocks, ptr<void>(aux_out), stream()),
           "gemm_colsum");
  return blocks;
}

// Adam descriptors for fused weight-gradient epilogues.  st = [p, m, v, shadow] per problem
// + the device step counter last; hp = [lr, b1, b2, eps, wd, decoupled].  Each state tensor
// must be laid out exactly like the gradient it replaces (same numel, contiguous).
void adam_descs(const std::vector<at::Tensor>& st, const std::vector<double>& hp, const at::Tensor* const* grads,
                int nprob, FdAdamEpi* out) {
  TORCH_CHECK((int)st.size() == 4 * nprob + 1, "fused adam: expected ", 4 * nprob + 1, " state tensors");
  TORCH_CHECK(hp.size() == 6, "fused adam: hyper-parameters [lr, b1, b2, eps, wd, decoupled]");
  const at::Tensor& step = st.back();
  need(step, at::kInt, "adam step");
  for (int i = 0; i < nprob; ++i) {
    const int64_t n = grads[i]->numel();
    for (int k = 0; k < 3; ++k) {
      need(st[4 * i + k], at::kFloat, "adam state");
      TORCH_CHECK(st[4 * i + k].numel() == n, "fused adam: state size mismatch");
    }
    const at::Tensor& sh = st[4 * i + 3];
    if (sh.defined() && sh.numel() > 0) {
      need(sh, at::kBFloat16, "adam shadow");
      TORCH_CHECK(sh.numel() == n, "fused adam: shadow size mismatch");
    }
    FdAdamEpi& a = out[i];
    a.p = st[4 * i].data_ptr<float>();
    a.m = st[4 * i + 1].data_ptr<float>();
    a.v = st[4 * i + 2].data_ptr<float>();
    a.sh = (sh.defined() && sh.numel() > 0) ? reinterpret_cast<uint16_t*>(sh.data_ptr()) : nullptr;
    a.step = step.data_ptr<int>();
    a.lr = (float)hp[0]; a.b1 = (float)hp[1]; a.b2 = (float)hp[2]; a.eps = (float)hp[3]; a.wd = (float)hp[4];
    a.decoupled = hp[5] != 0.0 ? 1 : 0;
  }
}

// Weight gradient C[M][N] (+)= A^T B (fp32; split-K slabs in `workspace`, reduced by a second
// launch), optionally with Adam fused into the epilogue (one K split).
void gemm_dw(const at::Tensor& A, const at::Tensor& B, const at::Tensor& C, const at::Tensor& workspace,
             bool accumulate, const std::vector<at::Tensor>& adam, const std::vector<double>& hp) {
  need(A, at::kBFloat16, "A");
  need(B, at::kBFloat16, "B");
  need(C, at::kFloat, "C");
  need(workspace, at::kFloat, "workspace");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm_dw operands must be 2-D");
  const int64_t K = A.size(0), M = A.size(1), N = B.size(1);
  TORCH_CHECK(B.size(0) == K && C.size(0) == M && C.size(1) == N, "gemm_dw: shape mismatch");
  TORCH_CHECK(K % 64 == 0 && M % 128 == 0 && N % 64 == 0, "gemm_dw: K % 64, M % 128, N % 64 required");
  FdAdamEpi ad{};
  const at::Tensor* gs[1] = {&C};
  if (!adam.empty()) adam_descs(adam, hp, gs, 1, &ad);
  check_rc(fd_gemm(2, 5, A.data_ptr(), B.data_ptr(), C.data_ptr(), (int)M, (int)N, (int)K, (int)M, (int)N, (int)N,
                   nullptr, nullptr, 0, nullptr, 0, workspace.data_ptr<float>(), workspace.numel(),
                   accumulate ? 1 : 0, adam.empty() ? nullptr : &ad, nullptr, nullptr, stream()),
           "gemm_dw");
}

// Grouped weight gradients: C0 (+)= A0^T B0 and C1 (+)= A1^T B1 in one launch (shared K = tokens).
int64_t gemm_dw2(const at::Tensor& A0, const at::Tensor& B0, const at::Tensor& C0, const at::Tensor& A1,
                 const at::Tensor& B1, const at::Tensor& C1, const at::Tensor& workspace, bool accumulate,
                 const std::vector<at::Tensor>& adam, const std::vector<double>& hp, bool defer) {
  const at::Tensor* As[2] = {&A0, &A1};
  const at::Tensor* Bs[2] = {&B0, &B1};
  const at::Tensor* Cs[2] = {&C0, &C1};
  const int64_t K = A0.size(0);
  for (int i = 0; i < 2; ++i) {
    need(*As[i], at::kBFloat16, "A");
    need(*Bs[i], at::kBFloat16, "B");
    need(*Cs[i], at::kFloat, "C");
    TORCH_CHECK(As[i]->dim() == 2 && Bs[i]->dim() == 2 && Cs[i]->dim() == 2, "gemm_dw2 operands must be 2-D");
    TORCH_CHECK(As[i]->size(0) == K && Bs[i]->size(0) == K, "gemm_dw2: all operands need K = ", K, " rows");
    TORCH_CHECK(Cs[i]->size(0) == As[i]->size(1) && Cs[i]->size(1) == Bs[i]->size(1), "gemm_dw2: C shape mismatch");
    TORCH_CHECK(As[i]->size(1) % 128 == 0 && Bs[i]->size(1) % 64 == 0, "gemm_dw2: M % 128 and N % 64 required");
  }
  TORCH_CHECK(K % 64 == 0, "gemm_dw2: K must be a multiple of 64");
  need(workspace, at::kFloat, "workspace");
  FdAdamEpi ad[2]{};
  if (!adam.empty()) adam_descs(adam, hp, Cs, 2, ad);
  int splits = 0;
  check_rc(fd_gemm_dw2(A0.data_ptr(), B0.data_ptr(), C0.data_ptr<float>(), (int)A0.size(1), (int)B0.size(1),
                       A1.data_ptr(), B1.data_ptr(), C1.data_ptr<float>(), (int)A1.size(1), (int)B1.size(1), (int)K,
                       workspace.data_ptr<float>(), workspace.numel(), accumulate ? 1 : 0,
                       adam.empty() ? nullptr : ad, defer ? 1 : 0, &splits, stream()),
           "gemm_dw2");
  return splits;  // > 0: slabs left in `workspace` (problem 0 then 1) for splitk_reduce_batched
}

// Every weight gradient of a backward in one launch (gemm.hip gemm_dw_batch_kernel):
// Cs[i] (+)= As[i]^T Bs[i] (fp32), As[i] [K_i][M_i], Bs[i] [K_i][N_i] bf16 (K_i % 64 == 0).
// adam: empty, or [p, m, v, shadow] per problem + the device step counter last (fused
// optimizer step instead of storing the gradients; hp = [lr, b1, b2, eps, wd, decoupled]).
void gemm_dw_batch(const std::vector<at::Tensor>& As, const std::vector<at::Tensor>& Bs,
                   const std::vector<at::Tensor>& Cs, const std::vector<int64_t>& accumulate,
                   const std::vector<at::Tensor>& adam, const std::vector<double>& hp, int64_t cfg,
                   const std::vector<at::Tensor>& biases = {}, const std::vector<at::Tensor>& rest = {},
                   const std::vector<int64_t>& rest_i = {}) {
  // biases: empty, or per problem an fp32 [M] producer-bias gradient (+)= column sums of A (an
  // empty tensor: none), accumulated like the problem's gradient
  // rest (with adam): the rest of the optimizer step in the same launch (FdAdamRest) -- [master,
  // grad, m, v, shadow] arenas, the run table (int64 [nruns][3]) and optionally the word table's
  // [ever, now] flags; rest_i = [n4 of the run table, word offset, word rows, word row length]
  const size_t n = As.size();
  TORCH_CHECK(n > 0 && n <= 32, "gemm_dw_batch: 1..32 problems, got ", n);
  TORCH_CHECK(Bs.size() == n && Cs.size() == n && accumulate.size() == n, "gemm_dw_batch: ragged problem lists");
  const int64_t K = As[0].size(0);
  std::vector<const at::Tensor*> cs(n);
  std::vector<FdDwProb> pr(n);
  for (size_t i = 0; i < n; ++i) {
    need(As[i], at::kBFloat16, "A");
    need(Bs[i], at::kBFloat16, "B");
    need(Cs[i], at::kFloat, "C");
    TORCH_CHECK(As[i].dim() == 2 && Bs[i].dim() == 2 && Cs[i].dim() == 2, "gemm_dw_batch operands must be 2-D");
    const int64_t Ki = As[i].size(0);
    TORCH_CHECK(Ki > 0 && Ki % 64 == 0, "gemm_dw_batch: K (rows) must be a positive multiple of 64, got ", Ki);
    TORCH_CHECK(Bs[i].size(0) == Ki, "gemm_dw_batch: A and B of a problem need the same rows (", Ki, ")");
    TORCH_CHECK(Cs[i].size(0) == As[i].size(1) && Cs[i].size(1) == Bs[i].size(1), "gemm_dw_batch: C shape mismatch");
    TORCH_CHECK(As[i].size(1) % 128 == 0 && Bs[i].size(1) % 64 == 0, "gemm_dw_batch: M % 128 and N % 64 required");
    cs[i] = &Cs[i];
    FdDwProb& q = pr[i];
    q = FdDwProb{};
    q.A = reinterpret_cast<const uint16_t*>(As[i].data_ptr());
    q.B = reinterpret_cast<const uint16_t*>(Bs[i].data_ptr());
    q.C = Cs[i].data_ptr<float>();
    q.M = (int)As[i].size(1);
    q.N = (int)Bs[i].size(1);
    q.K = (int)Ki;
    q.accumulate = accumulate[i] ? 1 : 0;
  }
  TORCH_CHECK(biases.empty() || biases.size() == n, "gemm_dw_batch: one bias entry per problem");
  for (size_t i = 0; i < biases.size(); ++i) {
    if (!biases[i].defined() || biases[i].numel() == 0) continue;
    need(biases[i], at::kFloat, "bias");
    TORCH_CHECK(biases[i].numel() == As[i].size(1), "gemm_dw_batch: a bias has the M entries of its problem");
    pr[i].bias = biases[i].data_ptr<float>();
  }
  std::vector<FdAdamEpi> ad(n);
  const int* step = nullptr;
  float hyper[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (!adam.empty()) {
    adam_descs(adam, hp, cs.data(), (int)n, ad.data());
    for (size_t i = 0; i < n; ++i) {
      TORCH_CHECK(!accumulate[i], "gemm_dw_batch: a fused Adam step cannot accumulate into a gradient");
      pr[i].p = ad[i].p; pr[i].m = ad[i].m; pr[i].v = ad[i].v; pr[i].sh = ad[i].sh;
    }
    step = ad[0].step;
    hyper[0] = ad[0].lr; hyper[1] = ad[0].b1; hyper[2] = ad[0].b2; hyper[3] = ad[0].eps; hyper[4] = ad[0].wd;
    hyper[5] = (float)ad[0].decoupled;
  }
  FdAdamRest rs{};
  if (!rest.empty()) {
    TORCH_CHECK(!adam.empty(), "gemm_dw_batch: the rest of the optimizer step needs the fused Adam");
    TORCH_CHECK((rest.size() == 6 || rest.size() == 8) && rest_i.size() == 4, "gemm_dw_batch: rest = 6 or 8 tensors, 4 ints");
    for (int k = 0; k < 4; ++k) need(rest[k], at::kFloat, "rest arena");
    need(rest[4], at::kBFloat16, "rest shadow");
    need(rest[5], at::kLong, "rest runs");
    const int64_t numel = rest[0].numel();
    for (int k = 1; k < 5; ++k) TORCH_CHECK(rest[k].numel() == numel, "gemm_dw_batch: rest arenas differ in size");
    TORCH_CHECK(rest[5].dim() == 2 && rest[5].size(1) == 3, "gemm_dw_batch: run table [n][3]");
    const int64_t n4 = rest_i[0], woff = rest_i[1], wrows = rest_i[2], wlen = rest_i[3];
    TORCH_CHECK(n4 >= 0 && n4 * 4 <= numel, "gemm_dw_batch: run table total out of range");
    rs.p = rest[0].data_ptr<float>(); rs.g = rest[1].data_ptr<float>(); rs.m = rest[2].data_ptr<float>();
    rs.v = rest[3].data_ptr<float>(); rs.sh = reinterpret_cast<uint16_t*>(rest[4].data_ptr());
    rs.runs = rest[5].size(0) ? reinterpret_cast<const long long*>(rest[5].data_ptr()) : nullptr;
    rs.nruns = (int)rest[5].size(0);
    rs.n4 = n4;
    if (rest.size() == 8) {
      need(rest[6], at::kByte, "rest ever");
      need(rest[7], at::kByte, "rest now");
      TORCH_CHECK(wlen > 0 && wlen % 4 == 0 && woff % 4 == 0 && woff >= 0 && woff + wrows * wlen <= numel &&
                      rest[6].numel() == wrows && rest[7].numel() == wrows,
                  "gemm_dw_batch: word table out of range");
      rs.ever = rest[6].data_ptr<unsigned char>(); rs.now = rest[7].data_ptr<unsigned char>();
      rs.woff = woff; rs.wrows = (int)wrows; rs.wrow4 = (int)(wlen / 4);
    }
    for (size_t i = 0; i < biases.size(); ++i)
      if (pr[i].bias) {
        const float* gb = rs.g;
        TORCH_CHECK(pr[i].bias >= gb && pr[i].bias + As[i].size(1) <= gb + numel,
                    "gemm_dw_batch: an in-launch bias Adam needs the bias gradient inside the grad arena");
      }
  }
  check_rc(fd_gemm_dw_batch((int)n, pr.data(), (int)K, step, adam.empty() ? nullptr : hyper, (int)cfg,
                            rest.empty() ? nullptr : &rs, stream()),
           "gemm_dw_batch");
}

// LayerNorm fused into the N = hidden NT GEMM C = A Bt^T (gemm.hip gemm_ln_kernel, FdLnEpi):
//   bwd = false: C = LN(dropout(A Bt^T + bias) + res) (gamma, beta), z = the bf16 pre-LN sum,
//                mean / rstd per row;
//   bwd = true:  dy = A Bt^T + res; C = dz (LN input gradient) from z, mean, rstd, gamma;
//                dx = dropout'(dz) (when thr); colpart[tiles_m][3][N] = dgamma, dbeta, dbias partials.
// stats (int64, >= 2 (M + 128) N / 64, zeroed once) is the row-statistic exchange, cnt (int32 [2],
// zeroed once) the exchange epoch (advanced per model forward by emb_fwd, or by the caller),
// err (int32) the timeout flag; xsite the launch's exchange call site (unique per epoch).
// Returns the number of row blocks (colpart rows).
int64_t gemm_ln(bool bwd, const at::Tensor& A, const at::Tensor& Bt, const at::Tensor& C,
                const c10::optional<at::Tensor>& bias, const at::Tensor& res, const at::Tensor& gamma,
                const c10::optional<at::Tensor>& beta, const at::Tensor& mean, const at::Tensor& rstd,
                const c10::optional<at::Tensor>& z, const c10::optional<at::Tensor>& dx,
                const c10::optional<at::Tensor>& colpart, const at::Tensor& stats, const at::Tensor& cnt,
                const at::Tensor& err, double eps, const c10::optional<at::Tensor>& seed, int64_t site, int64_t thr,
                double dscale, const c10::optional<at::Tensor>& row_map, int64_t cfg, int64_t xsite,
                bool b_mn = false, const c10::optional<at::Tensor>& xbuf = c10::nullopt,
                const c10::optional<at::Tensor>& prefetch = c10::nullopt) {
  // prefetch: the NEXT launch's weight operand (any dtype, contiguous), touched by the LayerNorm
  // epilogue while it waits for the row statistics (FdLnEpi::pf)
  // b_mn: Bt is the weight itself, W [K][N] (MN-major B through the LDS-DMA ring, transposing fragment reads)
  need(A, at::kBFloat16, "A");
  need(Bt, at::kBFloat16, "Bt");
  need(C, at::kBFloat16, "C");
  need(res, at::kBFloat16, "res");
  need(gamma, at::kFloat, "gamma");
  need(mean, at::kFloat, "mean");
  need(rstd, at::kFloat, "rstd");
  need(stats, at::kLong, "stats");
  need(cnt, at::kInt, "cnt");
  need(err, at::kInt, "err");
  TORCH_CHECK(A.dim() == 2 && Bt.dim() == 2 && C.dim() == 2 && res.dim() == 2, "gemm_ln operands must be 2-D");
  const int64_t M = A.size(0), K = A.size(1), N = b_mn ? Bt.size(1) : Bt.size(0);
  TORCH_CHECK(M > 0 && (b_mn ? Bt.size(0) : Bt.size(1)) == K && C.size(0) == M && C.size(1) == N,
              "gemm_ln: shape mismatch");
  TORCH_CHECK(res.size(0) == M && res.size(1) == N, "gemm_ln: res must be [M, N]");
  TORCH_CHECK(K % 64 == 0 && N % 64 == 0 && N <= 2048, "gemm_ln: K % 64, N % 64 and N <= 2048 required");
  TORCH_CHECK(gamma.numel() == N, "gemm_ln: gamma of size N required");
  TORCH_CHECK(mean.numel() >= M && rstd.numel() >= M, "gemm_ln: mean / rstd need M entries");
  TORCH_CHECK(stats.numel() >= 2 * (M + 128) * (N / 64), "gemm_ln: stats too small");
  TORCH_CHECK(cnt.numel() >= 1 && err.numel() >= 1, "gemm_ln: counters too small");
  // (xsite + 1 < FD_LN_XSITES: a granule tag epoch * FD_LN_XSITES + xsite + 1 is then never 0 mod
  // FD_LN_XSITES, so it can never equal the 0 of a granule zeroed at an epoch wrap)
  TORCH_CHECK(xsite >= 0 && xsite < FD_LN_XSITES - 1, "gemm_ln: exchange call site out of range");
  need_opt(bias, at::kFloat, "bias");
  need_opt(beta, at::kFloat, "beta");
  need_opt(z, at::kBFloat16, "z");
  need_opt(dx, at::kBFloat16, "dx");
  need_opt(colpart, at::kFloat, "colpart");
  need_opt(row_map, at::kInt, "row_map");
  const bool has_z = z.has_value() && z->defined();
  if (has_z) TORCH_CHECK(z->size(0) == M && z->size(1) == N, "gemm_ln: z must be [M, N]");
  if (!bwd) {
    TORCH_CHECK(bias.has_value() && bias->defined() && bias->numel() == N, "gemm_ln: bias of size N required");
    TORCH_CHECK(beta.has_value() && beta->defined() && beta->numel() == N, "gemm_ln: beta of size N required");
  } else {
    TORCH_CHECK(has_z, "gemm_ln backward needs the pre-LN sum z");
    TORCH_CHECK(colpart.has_value() && colpart->defined() && colpart->numel() >= ((M + 63) / 64) * 3 * N,
                "gemm_ln backward: colpart needs ceil(M/64) x 3N floats");
    if (thr) TORCH_CHECK(dx.has_value() && dx->defined() && dx->size(0) == M && dx->size(1) == N,
                         "gemm_ln backward with dropout needs dx [M, N]");
  }
  if (row_map.has_value() && row_map->defined()) TORCH_CHECK(row_map->numel() >= M, "gemm_ln: row_map needs M entries");
  FdLnEpi ln{};
  ln.gamma = gamma.data_ptr<float>();
  ln.beta = ptr<float>(beta);
  ln.mean = mean.data_ptr<float>();
  ln.rstd = rstd.data_ptr<float>();
  ln.z = ptr<uint16_t>(z);
  ln.dx = ptr<uint16_t>(dx);
  ln.colpart = ptr<float>(colpart);
  ln.stats = reinterpret_cast<uint64_t*>(stats.data_ptr());
  ln.cnt = cnt.data_ptr<int>();
  ln.err = err.data_ptr<int>();
  ln.eps = (float)eps;
  ln.thr = (uint32_t)thr;
  ln.site = (uint32_t)site;
  ln.dscale = (float)dscale;
  ln.xsite = (uint32_t)xsite;
  if (prefetch.has_value() && prefetch->defined() && prefetch->numel() > 0) {
    TORCH_CHECK(prefetch->is_cuda() == A.is_cuda() && prefetch->is_contiguous(), "gemm_ln: prefetch must be a contiguous device tensor");
    ln.pf = reinterpret_cast<const char*>(prefetch->data_ptr());
    ln.pf_bytes = (long long)(prefetch->numel() * prefetch->element_size());
  }
  if (thr) {
    TORCH_CHECK(seed.has_value() && seed->defined(), "gemm_ln: dropout needs the seed tensor");
    ln.seed_ptr = seedp(*seed);
    ln.row_map = ptr<int>(row_map);
  }
  // two-K-half tiles: the partial exchange (xbuf: >= tiles_m * N / 64 * 32 KiB) and its flag
  // granules, the last LN2_FLAGS entries of stats (zeroed with it at an epoch wrap)
  constexpr int64_t LN2_FLAGS = 512;
  if (xbuf.has_value() && xbuf->defined()) {
    need(*xbuf, at::kFloat, "xbuf");
    // (the launcher picks 128- or 256-row tiles: room for either)
    const int64_t pairs = ((M + 127) / 128) * (N / 128), pairs256 = ((M + 255) / 256) * (N / 128);
    if (xbuf->numel() >= std::max(pairs * 2 * 8192, pairs256 * 2 * 16384) && pairs * 2 <= LN2_FLAGS &&
        stats.numel() >= 2 * (M + 256) * (N / 64) + LN2_FLAGS) {
      ln.xbuf = xbuf->data_ptr<float>();
      ln.xflag = reinterpret_cast<uint64_t*>(stats.data_ptr()) + (stats.numel() - LN2_FLAGS);
    }
  }
  const int rc = fd_gemm_ln(bwd ? 1 : 0, A.data_ptr(), Bt.data_ptr(), C.data_ptr(), (int)M, (int)N, (int)K,
                            ptr<float>(bias), res.data_ptr(), (int)N, &ln, (int)cfg, b_mn ? 1 : 0, stream());
  TORCH_CHECK(rc > 0, "gemm_ln: kernel launcher rejected arguments (rc=", rc, ")");
  return rc;
}

// Split-K NT GEMM + fused epilogue (splitk.hip): C = epi(A Bt^T) through fp32 slabs in `workspace`.
// epi: 0 bf16, 1 bias, 2 bias+GELU (aux = u out), 3 GELU' (aux = u in, aux_out = gelu(u)), 4 residual,
// 6 LayerNorm forward, 7 LayerNorm backward (the ln_* arguments as for gemm_ln; colpart: M rows of
// [3][N]).  colsum (epi 3 / 4): ceil(M / 32) x N column partials of C.  Returns (splits, colsum
// partial rows).
std::vector<int64_t> gemm_splitk(int64_t epi, const at::Tensor& A, const at::Tensor& Bt, const at::Tensor& C,
                                 const at::Tensor& workspace, int64_t splits, const c10::optional<at::Tensor>& bias,
                                 const c10::optional<at::Tensor>& aux, const c10::optional<at::Tensor>& aux_out,
                                 const c10::optional<at::Tensor>& res, const c10::optional<at::Tensor>& colsum,
                                 const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
                                 const c10::optional<at::Tensor>& mean, const c10::optional<at::Tensor>& rstd,
                                 const c10::optional<at::Tensor>& z, const c10::optional<at::Tensor>& dx,
                                 const c10::optional<at::Tensor>& colpart, double eps,
                                 const c10::optional<at::Tensor>& seed, int64_t site, int64_t thr, double dscale,
                                 const c10::optional<at::Tensor>& row_map, bool b_mn = false,
                                 const std::vector<at::Tensor>& head = {}, const std::vector<double>& head_f = {},
                                 const c10::optional<at::Tensor>& head_dx = c10::nullopt,
                                 const c10::optional<at::Tensor>& head_tlogits = c10::nullopt,
                                 const c10::optional<at::Tensor>& head_own = c10::nullopt) {
  // b_mn: Bt is the weight W [K][N] itself (C = epi(A W); a dX GEMM without a W^T copy)
  need(A, at::kBFloat16, "A");
  need(Bt, at::kBFloat16, "Bt");
  need(C, at::kBFloat16, "C");
  need(workspace, at::kFloat, "workspace");
  TORCH_CHECK(A.dim() == 2 && Bt.dim() == 2 && C.dim() == 2, "gemm_splitk operands must be 2-D");
  const int64_t M = A.size(0), K = A.size(1), N = b_mn ? Bt.size(1) : Bt.size(0);
  TORCH_CHECK(M > 0 && (b_mn ? Bt.size(0) : Bt.size(1)) == K && C.size(0) == M && C.size(1) == N,
              "gemm_splitk: shape mismatch");
  TORCH_CHECK(K % 64 == 0 && N % 64 == 0, "gemm_splitk: K % 64 and N % 64 required");
  TORCH_CHECK(epi >= 0 && epi <= 7 && epi != 5, "gemm_splitk: epilogue code");
  for (const auto* t : {&aux, &aux_out, &res, &z, &dx}) {
    need_opt(*t, at::kBFloat16, "gemm_splitk bf16 operand");
    if (t->has_value() && (*t)->defined())
      TORCH_CHECK((*t)->dim() == 2 && (*t)->size(0) == M && (*t)->size(1) == N, "gemm_splitk: [M, N] operand");
  }
  for (const auto* t : {&bias, &gamma, &beta}) {
    need_opt(*t, at::kFloat, "gemm_splitk fp32 vector");
    if (t->has_value() && (*t)->defined()) TORCH_CHECK((*t)->numel() == N, "gemm_splitk: vector of size N");
  }
  need_opt(mean, at::kFloat, "mean");
  need_opt(rstd, at::kFloat, "rstd");
  need_opt(colsum, at::kFloat, "colsum");
  need_opt(colpart, at::kFloat, "colpart");
  need_opt(row_map, at::kInt, "row_map");
  auto has = [](const c10::optional<at::Tensor>& t) { return t.has_value() && t->defined(); };
  if (epi == 1 || epi == 2 || epi == 6) TORCH_CHECK(has(bias), "gemm_splitk: bias required");
  if (epi == 2 || epi == 3) TORCH_CHECK(has(aux), "gemm_splitk: aux [M, N] required");
  if (epi == 4 || epi >= 6) TORCH_CHECK(has(res), "gemm_splitk: res [M, N] required");
  if (has(colsum)) {
    TORCH_CHECK(epi == 3 || epi == 4, "gemm_splitk: column sums only with the GELU' / residual epilogues");
    TORCH_CHECK(colsum->numel() >= ((M + 31) / 32) * N, "gemm_splitk: colsum needs ceil(M/32) x N floats");
  }
  FdLnEpi ln{};
  if (epi >= 6) {
    TORCH_CHECK(has(gamma) && has(mean) && has(rstd) && mean->numel() >= M && rstd->numel() >= M,
                "gemm_splitk LayerNorm: gamma, mean / rstd of M entries required");
    if (epi == 6) TORCH_CHECK(has(beta), "gemm_splitk LayerNorm forward: beta required");
    if (epi == 7) {
      TORCH_CHECK(has(z), "gemm_splitk LayerNorm backward: z required");
      TORCH_CHECK(has(colpart) && colpart->numel() >= M * 3 * N, "gemm_splitk LayerNorm backward: colpart M x 3N");
      if (thr) TORCH_CHECK(has(dx), "gemm_splitk LayerNorm backward with dropout: dx required");
    }
    ln.gamma = gamma->data_ptr<float>();
    ln.beta = ptr<float>(beta);
    ln.mean = mean->data_ptr<float>();
    ln.rstd = rstd->data_ptr<float>();
    ln.z = ptr<uint16_t>(z);
    ln.dx = ptr<uint16_t>(dx);
    ln.colpart = ptr<float>(colpart);
    ln.eps = (float)eps;
    ln.thr = (uint32_t)thr;
    ln.site = (uint32_t)site;
    ln.dscale = (float)dscale;
    if (thr) {
      TORCH_CHECK(seed.has_value() && seed->defined(), "gemm_splitk: dropout needs the seed tensor");
      ln.seed_ptr = seedp(*seed);
      ln.row_map = ptr<int>(row_map);
      if (has(row_map)) TORCH_CHECK(row_map->numel() >= M, "gemm_splitk: row_map needs M entries");
    }
  }
  // the pruned step's head fused into the output-LayerNorm epilogue (splitk.hip sk_head_row):
  // head = [W [2][N], bias [2], labels [B] int64, logits [B][2], dlogits [B][2], dz [M][N] bf16,
  // colpart [M][3][N], hpart [M][2][N], dbpart [M][2], lpart [M], head seed int32, loss [1] fp32,
  // ticket [1] int32 (zeroed once; splitk.hip sk_head_row)],
  // head_f = [site, thr, dscale, kd_T, kd_alpha, B]
  FdSkHead hd{};
  if (!head.empty()) {
    TORCH_CHECK(epi == 6 && N == 768 && head.size() == 13 && head_f.size() == 6, "gemm_splitk head: arguments");
    need(head[11], at::kFloat, "head loss");
    need(head[12], at::kInt, "head ticket");
    TORCH_CHECK(head[11].numel() == 1 && head[12].numel() == 1, "gemm_splitk head: loss / ticket [1]");
    const int64_t Bh = (int64_t)head_f[5];
    TORCH_CHECK(Bh > 0 && Bh <= M, "gemm_splitk head: B");
    need(head[0], at::kFloat, "head W");
    need(head[1], at::kFloat, "head bias");
    need(head[2], at::kLong, "head labels");
    for (int k : {3, 4, 6, 7, 8, 9}) need(head[k], at::kFloat, "head fp32 output");
    need(head[5], at::kBFloat16, "head dz");
    TORCH_CHECK(head[0].numel() == 2 * N && head[1].numel() == 2 && head[2].numel() == Bh &&
                    head[3].numel() == 2 * Bh && head[4].numel() == 2 * Bh && head[5].numel() == M * N &&
                    head[6].numel() >= M * 3 * N && head[7].numel() >= M * 2 * N && head[8].numel() >= M * 2 &&
                    head[9].numel() >= M,
                "gemm_splitk head: sizes");
    need_opt(head_dx, at::kBFloat16, "head dx");
    need_opt(head_tlogits, at::kFloat, "head teacher logits");
    need_opt(head_own, at::kInt, "head own");
    if (thr) TORCH_CHECK(head_dx.has_value() && head_dx->defined() && head_dx->numel() == M * N, "gemm_splitk head: dx");
    if (head_tlogits.has_value() && head_tlogits->defined())
      TORCH_CHECK(head_tlogits->numel() == 2 * Bh && head_f[3] > 0.0, "gemm_splitk head: teacher logits [B, 2], T > 0");
    if (head_own.has_value() && head_own->defined()) TORCH_CHECK(head_own->numel() == Bh + 1, "gemm_splitk head: own");
    hd.W = head[0].data_ptr<float>();
    hd.bias = head[1].data_ptr<float>();
    hd.labels = reinterpret_cast<const long long*>(head[2].data_ptr());
    hd.logits = head[3].data_ptr<float>();
    hd.dlogits = head[4].data_ptr<float>();
    hd.dz = reinterpret_cast<uint16_t*>(head[5].data_ptr());
    hd.colpart = head[6].data_ptr<float>();
    hd.hpart = head[7].data_ptr<float>();
    hd.dbpart = head[8].data_ptr<float>();
    hd.lpart = head[9].data_ptr<float>();
    hd.seed_ptr = seedp(head[10]);
    hd.loss = head[11].data_ptr<float>();
    hd.ticket = reinterpret_cast<unsigned*>(head[12].data_ptr<int>());
    hd.site = (uint32_t)head_f[0];
    hd.thr = (uint32_t)head_f[1];
    hd.dscale = (float)head_f[2];
    hd.kd_T = (float)head_f[3];
    hd.kd_alpha = (float)head_f[4];
    hd.B = (int)Bh;
    hd.dx = ptr<uint16_t>(head_dx);
    hd.tlogits = ptr<const float>(head_tlogits);
    hd.own = ptr<int>(head_own);
  }
  int blocks = 0;
  const int rc = fd_gemm_splitk((int)epi, A.data_ptr(), Bt.data_ptr(), (int)M, (int)N, (int)K,
                                workspace.data_ptr<float>(), workspace.numel(), (int)splits, ptr<float>(bias),
                                C.data_ptr(), ptr<void>(aux), ptr<void>(aux_out), ptr<void>(res), ptr<float>(colsum),
                                &blocks, epi >= 6 ? &ln : nullptr, head.empty() ? nullptr : &hd, b_mn ? 1 : 0,
                                stream());
  TORCH_CHECK(rc > 0, "gemm_splitk: launcher rejected arguments (rc=", rc, ")");
  return {rc, blocks};
}

// Finish deferred split-K weight gradients: out_i (+)= sum_z slabs_i[z] (z order), one launch.
void splitk_reduce_batched(const std::vector<at::Tensor>& slabs, const std::vector<at::Tensor>& outs,
                           const std::vector<int64_t>& splits, const std::vector<int64_t>& accumulate) {
  const size_t n = slabs.size();
  TORCH_CHECK(outs.size() == n && splits.size() == n && accumulate.size() == n, "splitk_reduce_batched: ragged");
  std::vector<const float*> sp(n);
  std::vector<float*> op(n);
  std::vector<long long> ne(n);
  std::vector<int> sl(n), ac(n);
  for (size_t i = 0; i < n; ++i) {
    need(slabs[i], at::kFloat, "slabs");
    need(outs[i], at::kFloat, "out");
    TORCH_CHECK(splits[i] >= 1 && outs[i].numel() % 4 == 0 && slabs[i].numel() >= splits[i] * outs[i].numel(),
                "splitk_reduce_batched: slab buffer smaller than splits x out");
    sp[i] = slabs[i].data_ptr<float>();
    op[i] = outs[i].data_ptr<float>();
    ne[i] = outs[i].numel();
    sl[i] = (int)splits[i];
    ac[i] = accumulate[i] ? 1 : 0;
  }
  if (n) check_rc(fd_splitk_reduce_batched((int)n, sp.data(), op.data(), ne.data(), sl.data(), ac.data(), stream()),
                  "splitk_reduce_batched");
}

// Unpadded-step layout in one launch: row_map [rows] int32, cu [B+1] int32, ids_packed [rows] int64.
// step / seed (optional int32 [1]): counters advanced by the same launch (the step counter kernel folded in)
void pack(const at::Tensor& mask, const at::Tensor& ids, const at::Tensor& row_map, const at::Tensor& cu,
          const at::Tensor& ids_packed, const c10::optional<at::Tensor>& step, const c10::optional<at::Tensor>& seed,
          const c10::optional<at::Tensor>& cls_rows, const c10::optional<at::Tensor>& cls_rmap) {
  need_opt(cls_rmap, at::kInt, "cls_rmap");  // [>= B]: padded row of packed row cu[b] (int32)
  need_opt(step, at::kInt, "step");
  need_opt(seed, at::kInt, "seed");
  need_opt(cls_rows, at::kLong, "cls_rows");  // [>= B]: row cu[b] of sequence b (int64)
  TORCH_CHECK(on_device(mask) && mask.is_contiguous() && on_device(ids) && ids.is_contiguous(), "pack: GPU inputs");
  TORCH_CHECK(mask.dim() == 2 && ids.sizes() == mask.sizes(), "pack: mask and ids must both be [B, S]");
  need(row_map, at::kInt, "row_map");
  need(cu, at::kInt, "cu");
  need(ids_packed, at::kLong, "ids_packed");
  const int64_t B = mask.size(0), S = mask.size(1);
  TORCH_CHECK(cu.numel() == B + 1 && ids_packed.numel() == row_map.numel() && row_map.numel() >= 1, "pack: sizes");
  if (cls_rows.has_value() && cls_rows->defined()) TORCH_CHECK(cls_rows->numel() >= B, "pack: cls_rows needs B entries");
  if (cls_rmap.has_value() && cls_rmap->defined()) TORCH_CHECK(cls_rmap->numel() >= B, "pack: cls_rmap needs B entries");
  check_rc(fd_pack(mask.data_ptr(), (int)mask.element_size(), ids.data_ptr(), (int)ids.element_size(), (int)B, (int)S,
                   (int)row_map.numel(), row_map.data_ptr<int>(), cu.data_ptr<int>(),
                   reinterpret_cast<long long*>(ids_packed.data_ptr()), ptr<int>(step), ptr<uint32_t>(seed),
                   cls_rows.has_value() && cls_rows->defined() ? reinterpret_cast<long long*>(cls_rows->data_ptr())
                                                               : nullptr,
                   ptr<int>(cls_rmap), stream()),
           "pack");
}

// Pruned last block: (oa, ob)[k] = (a, b)[idx[k]] for k < n (same-shape bf16 [*, D] pairs), one launch.
void gather_rows2(const at::Tensor& a, const at::Tensor& b, const at::Tensor& oa, const at::Tensor& ob,
                  const at::Tensor& idx) {
  for (const at::Tensor* t : {&a, &b, &oa, &ob}) need(*t, at::kBFloat16, "gather_rows2 operand");
  need(idx, at::kLong, "idx");
  TORCH_CHECK(a.dim() == 2 && a.sizes() == b.sizes() && oa.dim() == 2 && oa.sizes() == ob.sizes() &&
                  oa.size(1) == a.size(1) && oa.size(0) == idx.numel(), "gather_rows2: shapes");
  TORCH_CHECK((a.size(1) * 2) % 16 == 0, "gather_rows2: rows must be 16-byte multiples");
  // (the indices are device data: the kernel trusts 0 <= idx < rows; the model builds them from cu)
  check_rc(fd_gather_rows2(a.data_ptr(), b.data_ptr(), oa.data_ptr(), ob.data_ptr(),
                           reinterpret_cast<const long long*>(idx.data_ptr()), (int)idx.numel(), (int)(a.size(1) * 2),
                           stream()), "gather_rows2");
}

// Pruned last block: oa / ob [T, D] = 0 except rows idx[k] (k < nsrc, ascending) = a / b [k].
void scatter_rows2(const at::Tensor& a, const at::Tensor& b, const at::Tensor& oa, const at::Tensor& ob,
                   const at::Tensor& idx, int64_t nsrc) {
  for (const at::Tensor* t : {&a, &b, &oa, &ob}) need(*t, at::kBFloat16, "scatter_rows2 operand");
  need(idx, at::kLong, "idx");
  TORCH_CHECK(a.dim() == 2 && a.sizes() == b.sizes() && oa.dim() == 2 && oa.sizes() == ob.sizes() &&
                  oa.size(1) == a.size(1) && nsrc >= 0 && nsrc <= a.size(0) && nsrc <= idx.numel(),
              "scatter_rows2: shapes");
  TORCH_CHECK((a.size(1) * 2) % 16 == 0, "scatter_rows2: rows must be 16-byte multiples");
  check_rc(fd_scatter_rows2(a.data_ptr(), b.data_ptr(), oa.data_ptr(), ob.data_ptr(),
                            reinterpret_cast<const long long*>(idx.data_ptr()), (int)nsrc, (int)oa.size(0),
                            (int)(a.size(1) * 2), stream()), "scatter_rows2");
}

// ---------------------------------------------------------------- native RCCL communicator
int comm_dtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kDouble: return 2;
    case at::kLong: return 3;
    case at::kInt: return 4;
    default: TORCH_CHECK(false, "comm: unsupported dtype ", t.scalar_type());
  }
  return 0;
}
void comm_check(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " failed: ", fd_comm_last_error()); }

void comm_load(const std::string& path) { comm_check(fd_comm_load(path.c_str()), "comm_load"); }

at::Tensor comm_unique_id() {
  at::Tensor id = at::empty({fd_comm_unique_id_bytes()}, at::TensorOptions().dtype(at::kByte));
  comm_check(fd_comm_get_unique_id(id.data_ptr()), "ncclGetUniqueId");
  return id;
}
int64_t comm_init(int64_t nranks, int64_t rank, const at::Tensor& id) {
  TORCH_CHECK(!id.is_cuda() && id.scalar_type() == at::kByte && id.numel() == fd_comm_unique_id_bytes(),
              "comm_init: id must be the CPU uint8 tensor from comm_unique_id()");
  TORCH_CHECK(rank >= 0 && rank < nranks, "comm_init: bad rank");
  void* c = nullptr;
  comm_check(fd_comm_init(&c, (int)nranks, (int)rank, id.contiguous().data_ptr()), "ncclCommInitRank");
  return reinterpret_cast<int64_t>(c);
}
void comm_destroy(int64_t h) { comm_check(fd_comm_destroy(reinterpret_cast<void*>(h)), "ncclCommDestroy"); }
void comm_abort(int64_t h) { comm_check(fd_comm_abort(reinterpret_cast<void*>(h)), "ncclCommAbort"); }
// (code, message): 0 = healthy; else the RCCL error of the communicator's async state
std::tuple<int64_t, std::string> comm_async_error(int64_t h) {
  const int rc = fd_comm_async_error(reinterpret_cast<void*>(h));
  return {rc, rc ? std::string(fd_comm_last_error()) : std::string()};
}
// Bounded wait for the current stream (the collective just issued on it): (code, message) with
// code 0 = done, 1001 = timeout, 1002 = HIP error, else the RCCL async error.  Releases the GIL.
std::tuple<int64_t, std::string> comm_wait(int64_t h, int64_t timeout_ms) {
  TORCH_CHECK(h != 0, "comm_wait: communicator not initialised");
  const hipStream_t st = stream();
  int rc;
  {
    py::gil_scoped_release nogil;
    rc = fd_comm_wait(reinterpret_cast<void*>(h), st, (long long)timeout_ms);
  }
  return {rc, rc ? std::string(fd_comm_last_error()) : std::string()};
}
void comm_allreduce(int64_t h, const at::Tensor& t, int64_t op) {
  TORCH_CHECK(h != 0, "comm_allreduce: communicator not initialised");
  TORCH_CHECK(on_device(t) && t.is_contiguous(), "comm_allreduce: contiguous GPU tensor required");
  TORCH_CHECK(op >= 0 && op <= 2, "comm_allreduce: op must be 0 (sum), 1 (avg) or 2 (max)");
  comm_check(fd_comm_allreduce(reinterpret_cast<void*>(h), t.data_ptr(), t.data_ptr(), t.numel(), comm_dtype(t),
                               (int)op, stream()),
             "ncclAllReduce");
}
void comm_broadcast(int64_t h, const at::Tensor& t, int64_t root) {
  TORCH_CHECK(h != 0, "comm_broadcast: communicator not initialised");
  TORCH_CHECK(on_device(t) && t.is_contiguous(), "comm_broadcast: contiguous GPU tensor required");
  comm_check(fd_comm_broadcast(reinterpret_cast<void*>(h), t.data_ptr(), t.numel(), comm_dtype(t), (int)root,
                               stream()),
             "ncclBroadcast");
}
void comm_allgather(int64_t h, const at::Tensor& send, const at::Tensor& recv) {
  TORCH_CHECK(h != 0, "comm_allgather: communicator not initialised");
  TORCH_CHECK(on_device(send) && on_device(recv) && send.is_contiguous() && recv.is_contiguous(),
              "comm_allgather: contiguous GPU tensors required");
  TORCH_CHECK(send.scalar_type() == recv.scalar_type() && recv.numel() % send.numel() == 0,
              "comm_allgather: recv must hold nranks x send");
  comm_check(fd_comm_allgather(reinterpret_cast<void*>(h), send.data_ptr(), recv.data_ptr(), send.numel(),
                               comm_dtype(send), stream()),
             "ncclAllGather");
}

// dsts[i] = srcs[i]^T for a batch of bf16 matrices (one launch).

// Diagnostic builds (FD_GEMM_STAMPS): per-block phase stamps of the last one-round GEMM launch
// into `out` (CPU int64 [nblocks][8]); returns the blocks copied (-1: a normal build).
int64_t gemm_stamps(at::Tensor out) {
  TORCH_CHECK(!out.is_cuda() && out.scalar_type() == at::kLong && out.is_contiguous() && out.dim() == 2 &&
                  out.size(1) == 8, "gemm_stamps: CPU int64 [n][8]");
  return fd_gemm_stamps(reinterpret_cast<unsigned long long*>(out.data_ptr()), (int)out.size(0));
}

// Diagnostic builds (FD_ATTN_STAMPS): per-block phase stamps of the last S <= 128 attention launch.
int64_t attn_stamps(at::Tensor out) {
  TORCH_CHECK(!out.is_cuda() && out.scalar_type() == at::kLong && out.is_contiguous() && out.dim() == 2 &&
                  out.size(1) == 8, "attn_stamps: CPU int64 [n][8]");
  return fd_attn_stamps(reinterpret_cast<unsigned long long*>(out.data_ptr()), (int)out.size(0));
}

// Tuning hook: force GEMM configuration `cfg` (-1 = measured default) for a kind.
void gemm_set_cfg(int64_t kind, int64_t cfg, int64_t splits) {
  check_rc(fd_gemm_set_cfg((int)kind, (int)cfg, (int)splits), "gemm_set_cfg");
}

// Varlen (packed) mode: `cu` = int32 [B+1] sequence starts in the packed rows of qkv/ctx
// (sequence b = rows cu[b] .. cu[b+1]-1, at most S long); the kernels clamp every row
// read to its sequence and never write outside it.  The caller guarantees cu[B] <= rows
// (the device values cannot be read here without a sync).
void check_cu(const c10::optional<at::Tensor>& cu, int64_t B, int64_t rows_qkv, int64_t rows_ctx) {
  if (!(cu.has_value() && cu->defined())) return;
  need(*cu, at::kInt, "cu");
  TORCH_CHECK(cu->numel() == B + 1, "attention: cu must have B+1 entries");
  TORCH_CHECK(rows_qkv >= 1 && rows_qkv == rows_ctx, "attention: packed qkv/ctx row counts differ");
}

// Optional int32 [T] packed-row -> padded-row map (dropout-hash indexing only).
const int* map_ptr(const c10::optional<at::Tensor>& m, int64_t T) {
  if (!(m.has_value() && m->defined())) return nullptr;
  need(*m, at::kInt, "row_map");
  TORCH_CHECK(m->numel() == T, "row_map must have one entry per row");
  return m->data_ptr<int>();
}

// Dropout keep bits handed from the S <= 128 attention forward to its backward: int64
// [B * H * 128 * 2] (used only by the S <= 128 kernels with dropout; nullable).
// split 2: a varlen batch at S > 128 whose sequences all have <= 128 tokens (the S <= 128 kernels alone)
void check_dmask(const c10::optional<at::Tensor>& dmask, int64_t B, int64_t S, int64_t H, int64_t split = -1) {
  if (!dmask.has_value() || !dmask->defined()) return;
  need(*dmask, at::kLong, "dmask");
  TORCH_CHECK((S <= 128 || split == 2) && dmask->numel() == B * H * 256,
              "attention: dmask needs S <= 128 (or split 2) and B*H*256 words");
}

void attn_fwd(const at::Tensor& qkv, const at::Tensor& kbias, const at::Tensor& ctx, const at::Tensor& lse,
              int64_t B, int64_t S, int64_t H, const at::Tensor& seed, int64_t site, int64_t thr, double dscale,
              const c10::optional<at::Tensor>& cu, const c10::optional<at::Tensor>& dmask, int64_t q_live = 0,
              const c10::optional<at::Tensor>& cxc = c10::nullopt, const c10::optional<at::Tensor>& xc = c10::nullopt,
              const c10::optional<at::Tensor>& xres = c10::nullopt, int64_t split = -1) {
  need(qkv, at::kBFloat16, "qkv");
  TORCH_CHECK(q_live >= 0, "attention: q_live >= 0");
  TORCH_CHECK(split >= -1 && split <= 2, "attention: split in -1..2");
  const bool compact = cxc.has_value() && cxc->defined();
  int64_t Bp = 0;
  if (compact) {  // [CLS] rows of ctx and of the residual stream, compacted to [Bp, D]
    TORCH_CHECK(q_live == 1 && xc.has_value() && xres.has_value(), "attention: compact rows need q_live 1, xc, xres");
    need(*cxc, at::kBFloat16, "cxc");
    need(*xc, at::kBFloat16, "xc");
    need(*xres, at::kBFloat16, "xres");
    Bp = cxc->numel() / (H * 64);
    TORCH_CHECK(Bp >= B && cxc->numel() == Bp * H * 64 && xc->numel() == cxc->numel(), "attention: cxc/xc size");
    TORCH_CHECK(xres->numel() == ctx.numel(), "attention: xres size");
  }
  need(kbias, at::kFloat, "kbias");
  need(ctx, at::kBFloat16, "ctx");
  need(lse, at::kFloat, "lse");
  check_dmask(dmask, B, S, H, split);
  TORCH_CHECK(S % 64 == 0 && S <= 512, "attention: S must be a multiple of 64 and <= 512");
  const bool varlen = cu.has_value() && cu->defined();
  const int64_t rows = varlen ? qkv.numel() / (3 * H * 64) : B * S;
  TORCH_CHECK(qkv.numel() == rows * 3 * H * 64 && ctx.numel() == rows * H * 64, "attention: qkv/ctx size");
  TORCH_CHECK((varlen || kbias.numel() == B * S) && lse.numel() == B * H * S, "attention: kbias/lse size");
  check_cu(cu, B, rows, ctx.numel() / (H * 64));
  check_rc(fd_attn_fwd(qkv.data_ptr(), kbias.data_ptr<float>(), ctx.data_ptr(), lse.data_ptr<float>(), (int)B,
                       (int)S, (int)H, seedp(seed), (uint32_t)site, (uint32_t)thr, (float)dscale, ptr<int>(cu),
                       (int)rows, ptr<uint64_t>(dmask), (int)q_live, compact ? cxc->data_ptr() : nullptr,
                       compact ? xc->data_ptr() : nullptr, compact ? xres->data_ptr() : nullptr, (int)Bp, (int)split,
                       stream()),
           "attn_fwd");
}

// QKV projection + S <= 128 attention forward in ONE launch (gemm.hip gemm_attn_fwd_kernel):
// qkv = x w^T + bias, then attn_fwd's outputs.  The tiles hand off to the attention items through
// QA_FLAGS tagged granules just before the LN2_FLAGS tail of the LayerNorm exchange state `stats`
// (same epoch `cnt`, timeout flag `err`; xsite unique per launch within an epoch).
constexpr int64_t QA_FLAGS = 1024, QA_LN2_FLAGS = 512;
void gemm_attn_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, const at::Tensor& qkv,
                   const at::Tensor& kbias, const at::Tensor& ctx, const at::Tensor& lse, int64_t B, int64_t S,
                   int64_t H, const at::Tensor& seed, int64_t site, int64_t thr, double dscale,
                   const c10::optional<at::Tensor>& cu, const c10::optional<at::Tensor>& dmask, int64_t q_live,
                   const at::Tensor& stats, const at::Tensor& cnt, const at::Tensor& err, int64_t xsite,
                   const c10::optional<at::Tensor>& cxc = c10::nullopt, const c10::optional<at::Tensor>& xc = c10::nullopt,
                   const c10::optional<at::Tensor>& xres = c10::nullopt,
                   const c10::optional<at::Tensor>& prefetch = c10::nullopt, int64_t mode = 1, int64_t split = -1) {
  // mode 1: the projection's tiles hand off to the attention items (flags); mode 2: one block per
  // (sequence, head) projects its own Q / K / V tile into the attention's LDS images
  need(x, at::kBFloat16, "x");
  TORCH_CHECK(mode == 1 || mode == 2, "gemm_attn_fwd: mode 1 or 2");
  need(w, at::kBFloat16, "w");
  need(bias, at::kFloat, "bias");
  need(qkv, at::kBFloat16, "qkv");
  need(kbias, at::kFloat, "kbias");
  need(ctx, at::kBFloat16, "ctx");
  need(lse, at::kFloat, "lse");
  need(stats, at::kLong, "stats");
  need(cnt, at::kInt, "cnt");
  need(err, at::kInt, "err");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && qkv.dim() == 2, "gemm_attn_fwd: x, w, qkv must be 2-D");
  const int64_t M = x.size(0), K = x.size(1), D = H * 64, N = 3 * D;
  TORCH_CHECK(H > 0 && w.size(0) == N && w.size(1) == K && bias.numel() == N && qkv.size(0) == M && qkv.size(1) == N,
              "gemm_attn_fwd: w [3 H 64, K], bias [3 H 64], qkv [M, 3 H 64] required");
  TORCH_CHECK(M > 0 && K % 64 == 0, "gemm_attn_fwd: K must be a multiple of 64");
  const bool short_ok = split == 2 && mode == 2 && cu.has_value() && cu->defined();  // (sequences <= 128 tokens)
  TORCH_CHECK(S % 64 == 0 && (S <= 128 || (short_ok && S <= 512)) && B > 0,
              "gemm_attn_fwd: S must be 64 or 128 (or <= 512 with split 2, mode 2, varlen)");
  TORCH_CHECK(M * N * 2 < (int64_t(1) << 31), "gemm_attn_fwd: qkv must stay below 2 GiB (32-bit buffer offsets)");
  TORCH_CHECK(q_live >= 0, "gemm_attn_fwd: q_live >= 0");
  TORCH_CHECK(xsite >= 0 && xsite < FD_LN_XSITES - 1, "gemm_attn_fwd: exchange call site out of range");
  TORCH_CHECK(cnt.numel() >= 1 && err.numel() >= 1, "gemm_attn_fwd: counters too small");
  const int64_t ntiles = ((M + 127) / 128) * (N / 192);
  TORCH_CHECK(ntiles <= QA_FLAGS && stats.numel() >= QA_FLAGS + QA_LN2_FLAGS,
              "gemm_attn_fwd: more tiles than flag granules, or stats too small");
  const bool compact = cxc.has_value() && cxc->defined();
  int64_t Bp = 0;
  if (compact) {
    TORCH_CHECK(q_live == 1 && xc.has_value() && xres.has_value(), "gemm_attn_fwd: compact rows need q_live 1, xc, xres");
    need(*cxc, at::kBFloat16, "cxc");
    need(*xc, at::kBFloat16, "xc");
    need(*xres, at::kBFloat16, "xres");
    Bp = cxc->numel() / D;
    TORCH_CHECK(Bp >= B && cxc->numel() == Bp * D && xc->numel() == cxc->numel(), "gemm_attn_fwd: cxc/xc size");
    TORCH_CHECK(xres->numel() == ctx.numel(), "gemm_attn_fwd: xres size");
  }
  check_dmask(dmask, B, S, H, split);
  const bool varlen = cu.has_value() && cu->defined();
  const int64_t rows = varlen ? M : B * S;
  TORCH_CHECK(M == rows && ctx.numel() == rows * D, "gemm_attn_fwd: qkv/ctx rows");
  TORCH_CHECK((varlen || kbias.numel() == B * S) && lse.numel() == B * H * S, "gemm_attn_fwd: kbias/lse size");
  check_cu(cu, B, rows, rows);
  uint64_t* flags = reinterpret_cast<uint64_t*>(stats.data_ptr()) + (stats.numel() - QA_LN2_FLAGS - QA_FLAGS);
  set_prefetch(prefetch, x);
  check_rc(fd_gemm_attn_fwd(x.data_ptr(), w.data_ptr(), bias.data_ptr<float>(), qkv.data_ptr(), (int)M, (int)K,
                            kbias.data_ptr<float>(), ctx.data_ptr(), lse.data_ptr<float>(), (int)B, (int)S, (int)H,
                            seedp(seed), (uint32_t)site, (uint32_t)thr, (float)dscale, ptr<int>(cu), (int)rows,
                            ptr<uint64_t>(dmask), (int)q_live, compact ? cxc->data_ptr() : nullptr,
                            compact ? xc->data_ptr() : nullptr, compact ? xres->data_ptr() : nullptr, (int)Bp, flags,
                            (int)QA_FLAGS, cnt.data_ptr<int>(), (int)xsite, err.data_ptr<int>(), (int)mode, (int)split,
                            stream()),
           "gemm_attn_fwd");
}

// The S <= 128 attention backward that computes its own dO: dctx = dy w (the out-projection's dX:
// dy [rows, K], w [K, H 64] the weight itself) per (sequence, head), inside the launch
// (gemm.hip attn_bwd_proj_kernel).  Full-query backward only.
void attn_bwd_proj(const at::Tensor& qkv, const at::Tensor& kbias, const at::Tensor& ctx, const at::Tensor& lse,
                   const at::Tensor& dy, const at::Tensor& w, const at::Tensor& dqkv, int64_t B, int64_t S, int64_t H,
                   const at::Tensor& seed, int64_t site, int64_t thr, double dscale,
                   const c10::optional<at::Tensor>& cu, const c10::optional<at::Tensor>& dmask, int64_t splits = 1,
                   const c10::optional<at::Tensor>& dresc = c10::nullopt,
                   const c10::optional<at::Tensor>& dres = c10::nullopt, int64_t split = -1) {
  // splits: the K splits of the out-projection GEMM this stands in for (its summation order);
  // dresc / dres: the pruned block's compact [CLS] form (dy = the [CLS] rows [Bp, K]), as attn_bwd
  check_dmask(dmask, B, S, H, split);
  const bool compact = dresc.has_value() && dresc->defined();
  TORCH_CHECK(compact == (dres.has_value() && dres->defined()), "attn_bwd_proj: dresc and dres go together");
  need(qkv, at::kBFloat16, "qkv");
  need(kbias, at::kFloat, "kbias");
  need(ctx, at::kBFloat16, "ctx");
  need(lse, at::kFloat, "lse");
  need(dy, at::kBFloat16, "dy");
  need(w, at::kBFloat16, "w");
  need(dqkv, at::kBFloat16, "dqkv");
  const bool short_ok = split == 2 && cu.has_value() && cu->defined();
  TORCH_CHECK(S % 64 == 0 && (S <= 128 || (short_ok && S <= 512)) && B > 0 && H > 0,
              "attn_bwd_proj: S must be 64 or 128 (or <= 512 with split 2, varlen)");
  const int64_t D = H * 64;
  const bool varlen = cu.has_value() && cu->defined();
  const int64_t rows = varlen ? qkv.numel() / (3 * D) : B * S;
  TORCH_CHECK(qkv.numel() == rows * 3 * D && dqkv.numel() == qkv.numel() && ctx.numel() == rows * D,
              "attn_bwd_proj: qkv / dqkv / ctx size");
  TORCH_CHECK(dy.dim() == 2 && (compact ? dy.size(0) >= B : dy.size(0) == rows) && w.dim() == 2 &&
                  w.size(0) == dy.size(1) && w.size(1) == D,
              "attn_bwd_proj: dy [rows (compact: >= B), K] and w [K, H 64] required");
  TORCH_CHECK(dy.size(1) % 64 == 0 && splits >= 1 && (dy.size(1) / 64) % splits == 0,
              "attn_bwd_proj: K must be a multiple of 64 and of 64 splits");
  if (compact) {
    need(*dresc, at::kBFloat16, "dresc");
    need(*dres, at::kBFloat16, "dres");
    TORCH_CHECK(dresc->numel() == dy.size(0) * D && dres->numel() == rows * D, "attn_bwd_proj: dresc / dres size");
  }
  TORCH_CHECK(lse.numel() == B * H * S && (varlen || kbias.numel() == B * S), "attn_bwd_proj: stats");
  check_cu(cu, B, rows, rows);
  check_rc(fd_attn_bwd_proj(qkv.data_ptr(), kbias.data_ptr<float>(), ctx.data_ptr(), lse.data_ptr<float>(),
                            dy.data_ptr(), w.data_ptr(), (int)dy.size(0), (int)dy.size(1), (int)splits, dqkv.data_ptr(),
                            (int)B, (int)S, (int)H, seedp(seed), (uint32_t)site, (uint32_t)thr, (float)dscale,
                            ptr<int>(cu), (int)rows, ptr<uint64_t>(dmask), compact ? dresc->data_ptr() : nullptr,
                            compact ? dres->data_ptr() : nullptr, (int)split, stream()),
           "attn_bwd_proj");
}

void attn_bwd(const at::Tensor& qkv, const at::Tensor& kbias, const at::Tensor& ctx, const at::Tensor& lse,
              const at::Tensor& dctx, const at::Tensor& delta, const at::Tensor& dqkv, int64_t B, int64_t S, int64_t H,
              const at::Tensor& seed, int64_t site, int64_t thr, double dscale, const c10::optional<at::Tensor>& cu,
              const c10::optional<at::Tensor>& dmask, int64_t q_live = 0,
              const c10::optional<at::Tensor>& dresc = c10::nullopt, const c10::optional<at::Tensor>& dres = c10::nullopt,
              int64_t split = -1) {
  TORCH_CHECK(q_live >= 0, "attention: q_live >= 0");
  TORCH_CHECK(split >= -1 && split <= 2, "attention: split in -1..2");
  check_dmask(dmask, B, S, H, split);
  // compact [CLS] gradients: dctx and dresc are [Bp, D], dres is the full-layout [rows, D] output
  const bool compact = dresc.has_value() && dresc->defined();
  TORCH_CHECK(compact == (dres.has_value() && dres->defined()), "attention bwd: dresc and dres go together");
  need(qkv, at::kBFloat16, "qkv");
  need(kbias, at::kFloat, "kbias");
  need(ctx, at::kBFloat16, "ctx");
  need(lse, at::kFloat, "lse");
  need(dctx, at::kBFloat16, "dctx");
  need(delta, at::kFloat, "delta");
  need(dqkv, at::kBFloat16, "dqkv");
  TORCH_CHECK(S % 64 == 0 && S <= 512, "attention: S must be a multiple of 64 and <= 512");
  const bool varlen = cu.has_value() && cu->defined();
  const int64_t rows = varlen ? qkv.numel() / (3 * H * 64) : B * S;
  TORCH_CHECK(qkv.numel() == rows * 3 * H * 64 && dqkv.numel() == qkv.numel(), "attention bwd: qkv size");
  if (compact) {
    TORCH_CHECK(q_live == 1, "attention bwd: compact [CLS] gradients need q_live 1");
    need(*dresc, at::kBFloat16, "dresc");
    need(*dres, at::kBFloat16, "dres");
    TORCH_CHECK(dctx.numel() % (H * 64) == 0 && dctx.numel() / (H * 64) >= B && dresc->numel() == dctx.numel(),
                "attention bwd: compact dctx / dresc size");
    TORCH_CHECK(ctx.numel() == rows * H * 64 && dres->numel() == ctx.numel(), "attention bwd: ctx / dres size");
  } else {
    TORCH_CHECK(ctx.numel() == rows * H * 64 && dctx.numel() == ctx.numel(), "attention bwd: ctx size");
  }
  TORCH_CHECK(lse.numel() == B * H * S && delta.numel() == B * H * S && (varlen || kbias.numel() == B * S),
              "attention bwd: stats");
  check_cu(cu, B, rows, ctx.numel() / (H * 64));
  check_rc(fd_attn_bwd(qkv.data_ptr(), kbias.data_ptr<float>(), ctx.data_ptr(), lse.data_ptr<float>(),
                       dctx.data_ptr(), delta.data_ptr<float>(), dqkv.data_ptr(), (int)B, (int)S, (int)H,
                       seedp(seed), (uint32_t)site, (uint32_t)thr, (float)dscale, ptr<int>(cu), (int)rows,
                       ptr<uint64_t>(dmask), (int)q_live, compact ? dresc->data_ptr() : nullptr,
                       compact ? dres->data_ptr() : nullptr, (int)split, stream()),
           "attn_bwd");
}

void mask_to_bias(const at::Tensor& mask, const at::Tensor& bias) {
  TORCH_CHECK(on_device(mask) && mask.is_contiguous(), "mask must be a contiguous GPU tensor");
  need(bias, at::kFloat, "bias");
  TORCH_CHECK(mask.numel() == bias.numel(), "mask/bias size");
  check_rc(fd_mask_to_bias(mask.data_ptr(), (int)mask.element_size(), bias.data_ptr<float>(), (long)mask.numel(),
                           stream()),
           "mask_to_bias");
}

void ln_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& r, const at::Tensor& gamma, const at::Tensor& beta,
            const at::Tensor& y, const at::Tensor& mean, const at::Tensor& rstd, double eps, const at::Tensor& seed,
            int64_t site, int64_t thr, double dscale, const c10::optional<at::Tensor>& row_map) {
  need(x, at::kBFloat16, "x");
  need_opt(r, at::kBFloat16, "r");
  need(gamma, at::kFloat, "gamma");
  need(beta, at::kFloat, "beta");
  need(y, at::kBFloat16, "y");
  need(mean, at::kFloat, "mean");
  need(rstd, at::kFloat, "rstd");
  const int64_t D = gamma.numel(), T = x.numel() / D;
  TORCH_CHECK(D == 768 && x.numel() == T * D && y.numel() == x.numel() && mean.numel() == T && rstd.numel() == T,
              "ln_fwd: shapes (D must be 768)");
  if (r.has_value() && r->defined()) TORCH_CHECK(r->numel() == x.numel(), "ln_fwd: residual size");
  check_rc(fd_ln_fwd(x.data_ptr(), ptr<void>(r), gamma.data_ptr<float>(), beta.data_ptr<float>(), y.data_ptr(),
                     mean.data_ptr<float>(), rstd.data_ptr<float>(), (int)T, (int)D, (float)eps, seedp(seed),
                     (uint32_t)site, (uint32_t)thr, (float)dscale, map_ptr(row_map, T), stream()),
           "ln_fwd");
}

int64_t ln_bwd(const at::Tensor& dy, const at::Tensor& x, const c10::optional<at::Tensor>& r, const at::Tensor& gamma,
            const at::Tensor& mean, const at::Tensor& rstd, const at::Tensor& dz, const c10::optional<at::Tensor>& dx,
            const c10::optional<at::Tensor>& dgamma, const c10::optional<at::Tensor>& dbeta,
            const c10::optional<at::Tensor>& dbias, const at::Tensor& work, const at::Tensor& seed, int64_t site,
            int64_t thr, double dscale, bool accumulate, const c10::optional<at::Tensor>& row_map, bool defer,
            bool zin) {
  // returns the number of [3][D] partial rows written to `work` (a deferred colsum job reduces them);
  // zin: x is the saved pre-LN sum z (fused-LN forward), no residual
  TORCH_CHECK(!zin || !(r.has_value() && r->defined()), "ln_bwd: zin takes no residual");
  need(dy, at::kBFloat16, "dy");
  need(x, at::kBFloat16, "x");
  need_opt(r, at::kBFloat16, "r");
  need(gamma, at::kFloat, "gamma");
  need(mean, at::kFloat, "mean");
  need(rstd, at::kFloat, "rstd");
  need(dz, at::kBFloat16, "dz");
  need_opt(dx, at::kBFloat16, "dx");
  need_opt(dgamma, at::kFloat, "dgamma");
  need_opt(dbeta, at::kFloat, "dbeta");
  need_opt(dbias, at::kFloat, "dbias");
  need(work, at::kFloat, "work");
  const int64_t D = gamma.numel(), T = x.numel() / D;
  TORCH_CHECK(D == 768 && dy.numel() == T * D && dz.numel() == T * D, "ln_bwd: shapes");
  TORCH_CHECK(work.numel() >= std::min<int64_t>(512, (T + 7) / 8) * 3 * D, "ln_bwd: work too small");
  if (thr != 0) TORCH_CHECK(dx.has_value() && dx->numel() == T * D, "ln_bwd: dx required with dropout");
  int nblk = 0;
  check_rc(fd_ln_bwd(dy.data_ptr(), x.data_ptr(), ptr<void>(r), gamma.data_ptr<float>(), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), dz.data_ptr(), ptr<void>(dx), ptr<float>(dgamma), ptr<float>(dbeta),
                     ptr<float>(dbias), work.data_ptr<float>(), (int)T, (int)D, seedp(seed), (uint32_t)site,
                     (uint32_t)thr, (float)dscale, accumulate ? 1 : 0, map_ptr(row_map, T), defer ? 1 : 0, &nblk,
                     zin ? 1 : 0, stream()),
           "ln_bwd");
  return nblk;
}

void emb_fwd(const at::Tensor& ids, const at::Tensor& word, const at::Tensor& pos, const at::Tensor& gamma,
             const at::Tensor& beta, const at::Tensor& y, const at::Tensor& mean, const at::Tensor& rstd, int64_t S,
             double eps, const at::Tensor& seed, int64_t site, int64_t thr, double dscale,
             const c10::optional<at::Tensor>& row_map, const c10::optional<at::Tensor>& ln_epoch,
             const c10::optional<at::Tensor>& sorted, const c10::optional<at::Tensor>& perm,
             const c10::optional<at::Tensor>& ln_stats) {
  TORCH_CHECK(on_device(ids) && ids.is_contiguous() && (ids.scalar_type() == at::kLong || ids.scalar_type() == at::kInt),
              "ids must be contiguous GPU int64/int32");
  // optional: the backward's id grouping (rank sort) computed by extra blocks of this launch
  need_opt(sorted, at::kLong, "sorted");
  need_opt(perm, at::kLong, "perm");
  const bool sort = sorted.has_value() && sorted->defined();
  TORCH_CHECK(sort == (perm.has_value() && perm->defined()), "emb_fwd: sorted and perm go together");
  if (sort)
    TORCH_CHECK(sorted->numel() == ids.numel() && perm->numel() == ids.numel() && ids.numel() <= 16384,
                "emb_fwd: sorted / perm need ids.numel() (<= 16384) elements");
  need_opt(ln_epoch, at::kInt, "ln_epoch");
  need_opt(ln_stats, at::kLong, "ln_stats");
  const bool has_stats = ln_stats.has_value() && ln_stats->defined();
  TORCH_CHECK(!has_stats || (ln_epoch.has_value() && ln_epoch->defined() && ln_stats->numel() > 0),
              "emb_fwd: ln_stats needs ln_epoch");
  need(word, at::kBFloat16, "word");
  need(pos, at::kBFloat16, "pos");
  need(gamma, at::kFloat, "gamma");
  need(beta, at::kFloat, "beta");
  need(y, at::kBFloat16, "y");
  const int64_t D = gamma.numel(), T = ids.numel();
  TORCH_CHECK(D == 768 && word.size(1) == D && pos.size(1) == D && y.numel() == T * D, "emb_fwd: shapes");
  const bool packed = row_map.has_value() && row_map->defined();
  TORCH_CHECK(S <= pos.size(0) && (packed || T % S == 0), "emb_fwd: S exceeds position table");
  check_rc(fd_emb_fwd(ids.data_ptr(), ids.scalar_type() == at::kLong, word.data_ptr(), pos.data_ptr(),
                      gamma.data_ptr<float>(), beta.data_ptr<float>(), y.data_ptr(), mean.data_ptr<float>(),
                      rstd.data_ptr<float>(), (int)T, (int)S, (int)D, (float)eps, seedp(seed), (uint32_t)site,
                      (uint32_t)thr, (float)dscale, map_ptr(row_map, T), ptr<int>(ln_epoch),
                      reinterpret_cast<unsigned long long*>(ptr<long long>(ln_stats)),
                      has_stats ? (long long)ln_stats->numel() : 0ll, ptr<long long>(sorted),
                      ptr<long long>(perm), stream()),
           "emb_fwd");
}

// Validated host arrays of a deferred column-sum batch (ops/kernels.py colsum_flush jobs).
struct ColsumHost {
  std::vector<const float*> pp;
  std::vector<float*> op;
  std::vector<int> nb, sd, dd, no, ac;
};
ColsumHost colsum_prepare(const std::vector<at::Tensor>& parts,
                          const std::vector<std::vector<c10::optional<at::Tensor>>>& outs,
                          const std::vector<int64_t>& nblk, const std::vector<int64_t>& stride,
                          const std::vector<int64_t>& D, const std::vector<int64_t>& accumulate) {
  const size_t n = parts.size();
  TORCH_CHECK(outs.size() == n && nblk.size() == n && stride.size() == n && D.size() == n && accumulate.size() == n,
              "colsum_batched: ragged job lists");
  ColsumHost h;
  h.pp.resize(n);
  h.op.assign(3 * n, nullptr);
  h.nb.resize(n); h.sd.resize(n); h.dd.resize(n); h.no.resize(n); h.ac.resize(n);
  for (size_t i = 0; i < n; ++i) {
    need(parts[i], at::kFloat, "colsum part");
    TORCH_CHECK(outs[i].size() >= 1 && outs[i].size() <= 3, "colsum_batched: 1..3 outputs per job");
    TORCH_CHECK(stride[i] >= (int64_t)outs[i].size() * D[i] && parts[i].numel() >= nblk[i] * stride[i],
                "colsum_batched: partial buffer too small");
    for (size_t k = 0; k < outs[i].size(); ++k) {
      if (outs[i][k].has_value() && outs[i][k]->defined()) {
        need(*outs[i][k], at::kFloat, "colsum out");
        TORCH_CHECK(outs[i][k]->numel() == D[i], "colsum_batched: output size");
        h.op[3 * i + k] = outs[i][k]->data_ptr<float>();
      }
    }
    h.pp[i] = parts[i].data_ptr<float>();
    h.nb[i] = (int)nblk[i]; h.sd[i] = (int)stride[i]; h.dd[i] = (int)D[i];
    h.no[i] = (int)outs[i].size(); h.ac[i] = accumulate[i] ? 1 : 0;
  }
  return h;
}

void emb_bwd(const at::Tensor& dy, const at::Tensor& ids, const at::Tensor& sorted, const at::Tensor& perm,
             const at::Tensor& word, const at::Tensor& pos, const at::Tensor& gamma, const at::Tensor& mean,
             const at::Tensor& rstd, const at::Tensor& dword, const at::Tensor& dpos, const at::Tensor& dgamma,
             const at::Tensor& dbeta, const at::Tensor& dz_buf, const at::Tensor& work, int64_t S,
             const at::Tensor& seed, int64_t site, int64_t thr, double dscale, bool accumulate,
             const c10::optional<at::Tensor>& now, const c10::optional<at::Tensor>& ever,
             const c10::optional<at::Tensor>& row_map, const c10::optional<at::Tensor>& cu,
             const std::vector<at::Tensor>& cs_parts = {},
             const std::vector<std::vector<c10::optional<at::Tensor>>>& cs_outs = {},
             const std::vector<int64_t>& cs_nblk = {}, const std::vector<int64_t>& cs_stride = {},
             const std::vector<int64_t>& cs_D = {}, const std::vector<int64_t>& cs_acc = {}) {
  // cs_*: deferred column-sum jobs (colsum_batched's arguments, <= 32) finalised by extra blocks of
  // the embedding tail's first launch instead of a launch of their own
  TORCH_CHECK(cs_parts.size() <= 32, "emb_bwd: at most 32 column-sum jobs");
  ColsumHost cs = colsum_prepare(cs_parts, cs_outs, cs_nblk, cs_stride, cs_D, cs_acc);
  need_opt(now, at::kByte, "now");
  need_opt(ever, at::kByte, "ever");
  TORCH_CHECK(now.has_value() == ever.has_value(), "emb_bwd: now/ever go together");
  if (now.has_value() && now->defined())
    TORCH_CHECK(now->numel() == word.size(0) && ever->numel() == word.size(0), "emb_bwd: flag sizes");
  need(dy, at::kBFloat16, "dy");
  need(sorted, at::kLong, "sorted");
  need(perm, at::kLong, "perm");
  need(dword, at::kFloat, "dword");
  need(dpos, at::kFloat, "dpos");
  need(dgamma, at::kFloat, "dgamma");
  need(dbeta, at::kFloat, "dbeta");
  need(dz_buf, at::kFloat, "dz_buf");
  need(work, at::kFloat, "work");
  const int64_t D = gamma.numel(), T = ids.numel(), V = word.size(0), P = pos.size(0);
  TORCH_CHECK(sorted.numel() == T && perm.numel() == T && dy.numel() == T * D && dz_buf.numel() >= T * D, "emb_bwd: sizes");
  const bool packed = cu.has_value() && cu->defined();
  TORCH_CHECK(packed == (row_map.has_value() && row_map->defined()), "emb_bwd: row_map and cu go together");
  if (packed) need(*cu, at::kInt, "cu");
  TORCH_CHECK(S <= P && (packed || T % S == 0), "emb_bwd: S / layout");
  const int64_t nseq = packed ? cu->numel() - 1 : T / S;
  // work: [T][D] word-gradient pieces, then the [min(256, ceil(T / 8))][3][D] LayerNorm partials
  TORCH_CHECK(dword.numel() == V * D && dpos.numel() == P * D &&
                  work.numel() >= T * D + std::min<int64_t>(256, (T + 7) / 8) * 3 * D,
              "emb_bwd: grad/work sizes");
  check_rc(fd_emb_bwd(dy.data_ptr(), ids.data_ptr(), ids.scalar_type() == at::kLong,
                      reinterpret_cast<const long long*>(sorted.data_ptr()),
                      reinterpret_cast<const long long*>(perm.data_ptr()), word.data_ptr(), pos.data_ptr(),
                      gamma.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(), dword.data_ptr<float>(),
                      dpos.data_ptr<float>(), dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
                      dz_buf.data_ptr<float>(), work.data_ptr<float>(), (int)T, (int)S, (int)nseq, (int)P, (int)V,
                      (int)D, seedp(seed), (uint32_t)site, (uint32_t)thr, (float)dscale, accumulate ? 1 : 0,
                      ptr<unsigned char>(now), ptr<unsigned char>(ever), map_ptr(row_map, T), ptr<int>(cu),
                      (int)cs_parts.size(), cs.pp.data(), cs.op.data(), cs.nb.data(), cs.sd.data(), cs.dd.data(),
                      cs.no.data(), cs.ac.data(), stream()),
           "emb_bwd");
}

void rank_sort(const at::Tensor& ids, const at::Tensor& sorted, const at::Tensor& perm) {
  TORCH_CHECK(on_device(ids) && ids.is_contiguous() && (ids.scalar_type() == at::kLong || ids.scalar_type() == at::kInt),
              "ids must be contiguous GPU int64/int32");
  need(sorted, at::kLong, "sorted");
  need(perm, at::kLong, "perm");
  TORCH_CHECK(sorted.numel() == ids.numel() && perm.numel() == ids.numel() && ids.numel() <= 16384,
              "rank_sort: sizes (T <= 16384)");
  check_rc(fd_rank_sort(ids.data_ptr(), ids.scalar_type() == at::kLong, (int)ids.numel(),
                        reinterpret_cast<long long*>(sorted.data_ptr()), reinterpret_cast<long long*>(perm.data_ptr()),
                        stream()),
           "rank_sort");
}

// Returns the number of partial rows left in `work` (what a deferred job must reduce).
int64_t colsum_bf16(const at::Tensor& x, const at::Tensor& out, const at::Tensor& work, bool accumulate, bool defer) {
  need(x, at::kBFloat16, "x");
  need(out, at::kFloat, "out");
  need(work, at::kFloat, "work");
  const int64_t N = out.numel(), T = x.numel() / N;
  TORCH_CHECK(T * N == x.numel() && work.numel() >= ((T + 31) / 32) * N, "colsum: sizes");
  int nblk = 0;
  check_rc(fd_colsum_bf16(x.data_ptr(), (int)T, (int)N, out.data_ptr<float>(), work.data_ptr<float>(),
                          accumulate ? 1 : 0, defer ? 1 : 0, &nblk, stream()),
           "colsum_bf16");
  return nblk;
}

// Partials of many bf16 column sums in one launch: parts[i] ([ceil(T_i / 32)][N_i] fp32) of xs[i]
// ([T_i][N_i] bf16), bitwise colsum_bf16(defer=True) of each.  Returns the partial row counts.
std::vector<int64_t> colsum_bf16_batched(const std::vector<at::Tensor>& xs, const std::vector<at::Tensor>& parts,
                                         const std::vector<int64_t>& N) {
  const size_t n = xs.size();
  TORCH_CHECK(parts.size() == n && N.size() == n, "colsum_bf16_batched: ragged job lists");
  std::vector<const void*> xp(n);
  std::vector<float*> pp(n);
  std::vector<int> tt(n), nn(n);
  std::vector<int64_t> nblk(n);
  for (size_t i = 0; i < n; ++i) {
    need(xs[i], at::kBFloat16, "colsum x");
    need(parts[i], at::kFloat, "colsum part");
    TORCH_CHECK(N[i] > 0 && N[i] % 4 == 0 && xs[i].numel() % N[i] == 0, "colsum_bf16_batched: x is not [T][N]");
    const int64_t T = xs[i].numel() / N[i];
    TORCH_CHECK(T > 0 && parts[i].numel() >= ((T + 31) / 32) * N[i], "colsum_bf16_batched: partial buffer too small");
    TORCH_CHECK(xs[i].device() == xs[0].device() && parts[i].device() == xs[0].device(), "colsum_bf16_batched: devices");
    xp[i] = xs[i].data_ptr();
    pp[i] = parts[i].data_ptr<float>();
    tt[i] = (int)T;
    nn[i] = (int)N[i];
    nblk[i] = (T + 31) / 32;
  }
  if (n) check_rc(fd_colsum_bf16_batched((int)n, xp.data(), tt.data(), nn.data(), pp.data(), stream()),
                  "colsum_bf16_batched");
  return nblk;
}

// One launch finalising many deferred column sums: job i reduces parts[i] ([nblk][stride] fp32)
// into outs[i][k] (k < 3, fp32 [D] or None) = sum over blocks of columns k*D .. k*D+D-1.
void colsum_batched(const std::vector<at::Tensor>& parts, const std::vector<std::vector<c10::optional<at::Tensor>>>& outs,
                    const std::vector<int64_t>& nblk, const std::vector<int64_t>& stride, const std::vector<int64_t>& D,
                    const std::vector<int64_t>& accumulate) {
  ColsumHost h = colsum_prepare(parts, outs, nblk, stride, D, accumulate);
  const size_t n = parts.size();
  if (n == 0) return;
  check_rc(fd_colsum_batched((int)n, h.pp.data(), h.op.data(), h.nb.data(), h.sd.data(), h.dd.data(), h.no.data(),
                             h.ac.data(), stream()),
           "colsum_batched");
}

void head_fwd(const at::Tensor& hidden, int64_t B, int64_t S, const at::Tensor& W, const at::Tensor& bias,
              const at::Tensor& seed, int64_t site, int64_t thr, double dscale, const c10::optional<at::Tensor>& labels,
              const at::Tensor& logits, const c10::optional<at::Tensor>& loss, const c10::optional<at::Tensor>& dlogits,
              const c10::optional<at::Tensor>& row_loss, const c10::optional<at::Tensor>& cls,
              const c10::optional<at::Tensor>& tlogits, double kd_T, double kd_alpha,
              const c10::optional<at::Tensor>& loss_acc) {
  need_opt(loss_acc, at::kFloat, "loss_acc");
  if (loss_acc.has_value() && loss_acc->defined()) TORCH_CHECK(loss_acc->numel() >= 1, "head_fwd: loss_acc [1]");
  need_opt(row_loss, at::kFloat, "row_loss");
  need_opt(tlogits, at::kFloat, "teacher logits");
  if (tlogits.has_value() && tlogits->defined())
    TORCH_CHECK(tlogits->numel() == 2 * B && labels.has_value() && labels->defined() && kd_T > 0.0,
                "head_fwd: distillation needs teacher logits [B, 2], labels and a temperature > 0");
  need_opt(cls, at::kInt, "cls");
  need(hidden, at::kBFloat16, "hidden");
  need(W, at::kFloat, "W");
  need(bias, at::kFloat, "bias");
  need(logits, at::kFloat, "logits");
  need_opt(labels, at::kLong, "labels");
  need_opt(loss, at::kFloat, "loss");
  need_opt(dlogits, at::kFloat, "dlogits");
  const int64_t D = W.size(1);
  const bool packed = cls.has_value() && cls->defined();
  TORCH_CHECK(W.size(0) == 2 && hidden.numel() % D == 0 && (packed || hidden.numel() == B * S * D) &&
                  logits.numel() == B * 2 && (!packed || cls->numel() == B),
              "head_fwd: shapes");
  if (labels.has_value() && labels->defined())
    TORCH_CHECK(labels->numel() == B && loss.has_value() && dlogits.has_value() && dlogits->numel() == 2 * B &&
                    row_loss.has_value() && row_loss->numel() >= B,
                "head_fwd: labels needs loss/dlogits/row_loss");
  check_rc(fd_head_fwd(hidden.data_ptr(), (int)B, (int)S, (int)D, W.data_ptr<float>(), bias.data_ptr<float>(),
                       seedp(seed), (uint32_t)site, (uint32_t)thr, (float)dscale,
                       ptr<const long long>(labels), logits.data_ptr<float>(), ptr<float>(loss), ptr<float>(dlogits),
                       ptr<float>(row_loss), ptr<int>(cls), (int)(hidden.numel() / D), ptr<const float>(tlogits),
                       (float)kd_T, (float)kd_alpha, ptr<float>(loss_acc), stream()),
           "head_fwd");
}

void head_bwd(const at::Tensor& hidden, int64_t B, int64_t S, const at::Tensor& W, const at::Tensor& seed, int64_t site,
              int64_t thr, double dscale, const at::Tensor& dlogits, const at::Tensor& dW, const at::Tensor& db,
              const at::Tensor& dhidden, bool accumulate, const c10::optional<at::Tensor>& cls,
              const c10::optional<at::Tensor>& gscale, const c10::optional<at::Tensor>& own) {
  need_opt(cls, at::kInt, "cls");
  need_opt(gscale, at::kFloat, "gscale");
  need_opt(own, at::kInt, "own");
  if (own.has_value() && own->defined()) TORCH_CHECK(own->numel() == B + 1, "head_bwd: own must be [B + 1]");
  if (gscale.has_value() && gscale->defined()) TORCH_CHECK(gscale->numel() == 1, "head_bwd: gscale is a scalar");
  need(hidden, at::kBFloat16, "hidden");
  need(W, at::kFloat, "W");
  need(dlogits, at::kFloat, "dlogits");
  need(dW, at::kFloat, "dW");
  need(db, at::kFloat, "db");
  need(dhidden, at::kBFloat16, "dhidden");
  const int64_t D = W.size(1);
  const bool packed = cls.has_value() && cls->defined();
  TORCH_CHECK(hidden.numel() % D == 0 && (packed || hidden.numel() == B * S * D) && (!packed || cls->numel() == B) &&
                  dhidden.numel() == hidden.numel() && dlogits.numel() == 2 * B && dW.numel() == 2 * D &&
                  db.numel() == 2,
              "head_bwd: shapes");
  check_rc(fd_head_bwd(hidden.data_ptr(), (int)B, (int)S, (int)D, W.data_ptr<float>(), seedp(seed), (uint32_t)site,
                       (uint32_t)thr, (float)dscale, dlogits.data_ptr<float>(), dW.data_ptr<float>(),
                       db.data_ptr<float>(), dhidden.data_ptr(), accumulate ? 1 : 0, ptr<int>(cls),
                       (int)(hidden.numel() / D), ptr<float>(gscale), ptr<int>(own), stream()),
           "head_bwd");
}


// The pruned training step's head forward + backward + the last block's output-LayerNorm backward
// in one launch (norm.hip head_ln_bwd_kernel; the loss's upstream gradient is 1).  hidden / z /
// dz / dx [T][D] (head row b = hidden row b, b < B <= T); returns the partial rows written to
// `work` ([n][3][D] dgamma / dbeta / dbias, for a deferred column-sum job).
int64_t head_ln_bwd(const at::Tensor& hidden, int64_t B, const at::Tensor& W, const at::Tensor& bias,
                    const at::Tensor& seed, int64_t hsite, int64_t hthr, double hdscale, const at::Tensor& labels,
                    const at::Tensor& logits, const at::Tensor& loss, const at::Tensor& dlogits,
                    const at::Tensor& row_loss, const c10::optional<at::Tensor>& loss_acc, const at::Tensor& dW,
                    const at::Tensor& db, bool accumulate, const c10::optional<at::Tensor>& own,
                    const c10::optional<at::Tensor>& tlogits, double kd_T, double kd_alpha, const at::Tensor& z,
                    const at::Tensor& gamma, const at::Tensor& mean, const at::Tensor& rstd, const at::Tensor& dz,
                    const c10::optional<at::Tensor>& dx, const at::Tensor& work, int64_t site, int64_t thr,
                    double dscale, const c10::optional<at::Tensor>& row_map) {
  need(hidden, at::kBFloat16, "hidden");
  need(W, at::kFloat, "W");
  need(bias, at::kFloat, "bias");
  need(labels, at::kLong, "labels");
  need(logits, at::kFloat, "logits");
  need(loss, at::kFloat, "loss");
  need(dlogits, at::kFloat, "dlogits");
  need(row_loss, at::kFloat, "row_loss");
  need_opt(loss_acc, at::kFloat, "loss_acc");
  need(dW, at::kFloat, "dW");
  need(db, at::kFloat, "db");
  need_opt(own, at::kInt, "own");
  need_opt(tlogits, at::kFloat, "teacher logits");
  need(z, at::kBFloat16, "z");
  need(gamma, at::kFloat, "gamma");
  need(mean, at::kFloat, "mean");
  need(rstd, at::kFloat, "rstd");
  need(dz, at::kBFloat16, "dz");
  need_opt(dx, at::kBFloat16, "dx");
  need(work, at::kFloat, "work");
  const int64_t D = W.size(1);
  const int64_t T = hidden.numel() / std::max<int64_t>(D, 1);
  TORCH_CHECK(D == 768 && W.size(0) == 2 && gamma.numel() == D && bias.numel() == 2 && hidden.numel() == T * D,
              "head_ln_bwd: shapes");
  TORCH_CHECK(B > 0 && B <= T && B <= 1024, "head_ln_bwd: 0 < B <= min(T, 1024)");
  TORCH_CHECK(labels.numel() == B && logits.numel() == 2 * B && dlogits.numel() == 2 * B && loss.numel() == 1 &&
                  row_loss.numel() >= B && dW.numel() == 2 * D && db.numel() == 2,
              "head_ln_bwd: head outputs");
  TORCH_CHECK(z.numel() == T * D && dz.numel() == T * D && mean.numel() >= T && rstd.numel() >= T,
              "head_ln_bwd: LayerNorm operands");
  if (own.has_value() && own->defined()) TORCH_CHECK(own->numel() == B + 1, "head_ln_bwd: own must be [B + 1]");
  if (loss_acc.has_value() && loss_acc->defined()) TORCH_CHECK(loss_acc->numel() >= 1, "head_ln_bwd: loss_acc [1]");
  if (tlogits.has_value() && tlogits->defined())
    TORCH_CHECK(tlogits->numel() == 2 * B && kd_T > 0.0, "head_ln_bwd: teacher logits [B, 2], T > 0");
  if (thr != 0) TORCH_CHECK(dx.has_value() && dx->defined() && dx->numel() == T * D, "head_ln_bwd: dx required with dropout");
  TORCH_CHECK(work.numel() >= ((T + 15) / 16) * 3 * D, "head_ln_bwd: work too small");
  int nblk = 0;
  check_rc(fd_head_ln_bwd(hidden.data_ptr(), (int)B, (int)T, (int)D, W.data_ptr<float>(), bias.data_ptr<float>(),
                          seedp(seed), (uint32_t)hsite, (uint32_t)hthr, (float)hdscale,
                          reinterpret_cast<const long long*>(labels.data_ptr()), logits.data_ptr<float>(),
                          loss.data_ptr<float>(), dlogits.data_ptr<float>(), row_loss.data_ptr<float>(),
                          ptr<float>(loss_acc), dW.data_ptr<float>(), db.data_ptr<float>(), accumulate ? 1 : 0,
                          ptr<int>(own), ptr<const float>(tlogits), (float)kd_T, (float)kd_alpha, z.data_ptr(),
                          gamma.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(), dz.data_ptr(),
                          ptr<void>(dx), work.data_ptr<float>(), (uint32_t)site, (uint32_t)thr, (float)dscale,
                          map_ptr(row_map, T), &nblk, stream()),
           "head_ln_bwd");
  return nblk;
}

void eval_metrics(const at::Tensor& logits, const at::Tensor& labels, const at::Tensor& acc, const at::Tensor& counts,
                  const c10::optional<at::Tensor>& prob1, const c10::optional<at::Tensor>& preds) {
  need(logits, at::kFloat, "logits");
  need(labels, at::kLong, "labels");
  need(acc, at::kDouble, "acc");
  need(counts, at::kLong, "counts");
  need_opt(prob1, at::kFloat, "prob1");
  need_opt(preds, at::kLong, "preds");
  const int64_t B = labels.numel();
  TORCH_CHECK(logits.numel() == 2 * B && acc.numel() >= 1 && counts.numel() >= 5, "eval_metrics: shapes");
  check_rc(fd_eval_metrics(logits.data_ptr<float>(), reinterpret_cast<const long long*>(labels.data_ptr()), (int)B,
                           acc.data_ptr<double>(), reinterpret_cast<long long*>(counts.data_ptr()), ptr<float>(prob1),
                           ptr<long long>(preds), stream()),
           "eval_metrics");
}

void adam(const at::Tensor& p, const at::Tensor& g, const at::Tensor& m, const at::Tensor& v,
          const c10::optional<at::Tensor>& shadow, const at::Tensor& step, double lr, double b1, double b2, double eps,
          double wd, bool decoupled, const c10::optional<at::Tensor>& touched, const c10::optional<at::Tensor>& now,
          int64_t skip_off, int64_t skip_rows, int64_t row_len, const c10::optional<at::Tensor>& runs,
          int64_t run_total4, int64_t run_end4) {
  need_opt(touched, at::kByte, "touched");
  need_opt(now, at::kByte, "now");
  if (touched.has_value() && touched->defined()) {
    TORCH_CHECK(touched->numel() >= skip_rows && skip_off >= 0 && skip_off + skip_rows * row_len <= p.numel(),
                "adam: skip range");
    if (now.has_value() && now->defined()) TORCH_CHECK(now->numel() >= skip_rows, "adam: now size");
  }
  need(p, at::kFloat, "p");
  need(g, at::kFloat, "g");
  need(m, at::kFloat, "m");
  need(v, at::kFloat, "v");
  need_opt(shadow, at::kBFloat16, "shadow");
  need(step, at::kInt, "step");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n && n % 4 == 0, "adam: sizes");
  if (shadow.has_value() && shadow->defined()) TORCH_CHECK(shadow->numel() == n, "adam: shadow size");
  // run table [start4, count4, prefix4] x nruns (int64, on the device).  The caller built it on
  // the host (engine/optim.py) and passes its total and its largest end, checked here against
  // the arena so the kernel's indexing stays in bounds.
  const long long* rp = nullptr;
  int nruns = 0;
  long long total4 = 0;
  if (runs.has_value() && runs->defined()) {
    need(*runs, at::kLong, "adam runs");
    TORCH_CHECK(runs->dim() == 2 && runs->size(1) == 3 && runs->size(0) > 0, "adam runs: [nruns, 3]");
    TORCH_CHECK(run_total4 > 0 && run_end4 <= n / 4, "adam runs: total / end outside the arena");
    nruns = (int)runs->size(0);
    rp = reinterpret_cast<const long long*>(runs->data_ptr<int64_t>());
    total4 = run_total4;
  }
  check_rc(fd_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                   ptr<void>(shadow), n, step.data_ptr<int>(), (float)lr, (float)b1, (float)b2, (float)eps, (float)wd,
                   decoupled ? 1 : 0, ptr<const unsigned char>(touched), ptr<const unsigned char>(now), skip_off,
                   skip_rows, (int)row_len, rp, nruns, total4, stream()),
           "adam");
}

// Adam (weight decay 0) over the rows of a [rows][row_len] table whose `ever` flag is set
// (gradient taken as 0 unless now[row]); p, g, m, v (and shadow) are that table's views.
void adam_rows(const at::Tensor& p, const at::Tensor& g, const at::Tensor& m, const at::Tensor& v,
               const c10::optional<at::Tensor>& shadow, const at::Tensor& step, double lr, double b1, double b2,
               double eps, const at::Tensor& ever, const c10::optional<at::Tensor>& now, int64_t row_len) {
  need(p, at::kFloat, "p");
  need(g, at::kFloat, "g");
  need(m, at::kFloat, "m");
  need(v, at::kFloat, "v");
  need_opt(shadow, at::kBFloat16, "shadow");
  need(step, at::kInt, "step");
  need(ever, at::kByte, "ever");
  need_opt(now, at::kByte, "now");
  const int64_t n = p.numel();
  TORCH_CHECK(row_len > 0 && row_len % 4 == 0 && n % row_len == 0, "adam_rows: rows of row_len (multiple of 4)");
  const int64_t rows = n / row_len;
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adam_rows: sizes");
  if (shadow.has_value() && shadow->defined()) TORCH_CHECK(shadow->numel() == n, "adam_rows: shadow size");
  TORCH_CHECK(ever.numel() >= rows, "adam_rows: ever flags");
  if (now.has_value() && now->defined()) TORCH_CHECK(now->numel() >= rows, "adam_rows: now flags");
  check_rc(fd_adam_rows(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                        ptr<void>(shadow), (int)rows, (int)row_len, step.data_ptr<int>(), (float)lr, (float)b1,
                        (float)b2, (float)eps, ever.data_ptr<unsigned char>(), ptr<const unsigned char>(now),
                        stream()),
           "adam_rows");
}

void step_inc(const c10::optional<at::Tensor>& step, const c10::optional<at::Tensor>& seed) {
  need_opt(step, at::kInt, "step");
  need_opt(seed, at::kInt, "seed");
  check_rc(fd_step(ptr<int>(step), ptr<uint32_t>(seed), stream()), "step");
}

void scale_cast(const at::Tensor& p, const c10::optional<at::Tensor>& shadow, double scale) {
  need(p, at::kFloat, "p");
  need_opt(shadow, at::kBFloat16, "shadow");
  TORCH_CHECK(p.numel() % 4 == 0, "scale_cast: numel % 4");
  if (shadow.has_value() && shadow->defined()) TORCH_CHECK(shadow->numel() == p.numel(), "scale_cast: shadow size");
  check_rc(fd_scale_cast(p.data_ptr<float>(), ptr<void>(shadow), p.numel(), (float)scale, stream()), "scale_cast");
}

void axpby(const at::Tensor& dst, const at::Tensor& x, const c10::optional<at::Tensor>& y, double a, double b) {
  need(dst, at::kFloat, "dst");
  need(x, at::kFloat, "x");
  need_opt(y, at::kFloat, "y");
  TORCH_CHECK(dst.numel() == x.numel() && dst.numel() % 4 == 0, "axpby: sizes");
  if (y.has_value() && y->defined()) TORCH_CHECK(y->numel() == x.numel(), "axpby: y size");
  check_rc(fd_axpby(dst.data_ptr<float>(), x.data_ptr<float>(), ptr<const float>(y), (float)a, (float)b, dst.numel(),
                    stream()),
           "axpby");
}

}  // namespace

#ifndef FD_HOST_VALIDATION
PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 HIP kernels for the federated DistilBERT engine";
  m.def("gemm", &gemm, py::arg("kind"), py::arg("epi"), py::arg("A"), py::arg("B"), py::arg("C"), py::arg("bias"),
        py::arg("aux"), py::arg("res"), py::arg("workspace"), py::arg("accumulate"), py::arg("aux_out") = py::none(),
        py::arg("prefetch") = py::none());
  m.def("gemm_set_cfg", &gemm_set_cfg);
  m.def("gemm_stamps", &gemm_stamps);
  m.def("attn_stamps", &attn_stamps);
  m.def("gemm_splitk", &gemm_splitk, py::arg("epi"), py::arg("A"), py::arg("Bt"), py::arg("C"), py::arg("workspace"),
        py::arg("splits") = 0, py::arg("bias") = py::none(), py::arg("aux") = py::none(),
        py::arg("aux_out") = py::none(), py::arg("res") = py::none(), py::arg("colsum") = py::none(),
        py::arg("gamma") = py::none(), py::arg("beta") = py::none(), py::arg("mean") = py::none(),
        py::arg("rstd") = py::none(), py::arg("z") = py::none(), py::arg("dx") = py::none(),
        py::arg("colpart") = py::none(), py::arg("eps") = 1e-12, py::arg("seed") = py::none(),
        py::arg("site") = 0, py::arg("thr") = 0, py::arg("dscale") = 1.0, py::arg("row_map") = py::none(),
        py::arg("b_mn") = false, py::arg("head") = std::vector<at::Tensor>{}, py::arg("head_f") = std::vector<double>{},
        py::arg("head_dx") = py::none(), py::arg("head_tlogits") = py::none(), py::arg("head_own") = py::none());
  m.def("gemm_dw2", &gemm_dw2);
  m.def("gemm_dw", &gemm_dw);
  m.def("adam_rows", &adam_rows);
  m.def("gemm_ln", &gemm_ln, py::arg("bwd"), py::arg("A"), py::arg("Bt"), py::arg("C"), py::arg("bias"),
        py::arg("res"), py::arg("gamma"), py::arg("beta"), py::arg("mean"), py::arg("rstd"), py::arg("z"),
        py::arg("dx"), py::arg("colpart"), py::arg("stats"), py::arg("cnt"), py::arg("err"), py::arg("eps"),
        py::arg("seed"), py::arg("site"), py::arg("thr"), py::arg("dscale"), py::arg("row_map"),
        py::arg("cfg") = -1, py::arg("xsite") = 0, py::arg("b_mn") = false, py::arg("xbuf") = py::none(),
        py::arg("prefetch") = py::none());
  m.def("gemm_dw_batch", &gemm_dw_batch, py::arg("As"), py::arg("Bs"), py::arg("Cs"), py::arg("accumulate"),
        py::arg("adam"), py::arg("hp"), py::arg("cfg") = -1,
        py::arg("biases") = std::vector<at::Tensor>{}, py::arg("rest") = std::vector<at::Tensor>{},
        py::arg("rest_i") = std::vector<int64_t>{});
  m.def("gemm_colsum", &gemm_colsum, py::arg("epi"), py::arg("A"), py::arg("B"), py::arg("C"), py::arg("aux"),
        py::arg("res"), py::arg("colsum"), py::arg("aux_out") = py::none(), py::arg("kind") = 0,
        py::arg("prefetch") = py::none());
  m.def("splitk_reduce_batched", &splitk_reduce_batched);
  m.def("gemm_dw2_splits", [](int64_t M0, int64_t N0, int64_t M1, int64_t N1, int64_t K) {
    return (int64_t)fd_gemm_dw2_splits((int)M0, (int)N0, (int)M1, (int)N1, (int)K);
  });
  m.def("gather_rows2", &gather_rows2);
  m.def("scatter_rows2", &scatter_rows2);
  m.def("pack", &pack, py::arg("mask"), py::arg("ids"), py::arg("row_map"), py::arg("cu"), py::arg("ids_packed"),
        py::arg("step") = py::none(), py::arg("seed") = py::none(), py::arg("cls_rows") = py::none(),
        py::arg("cls_rmap") = py::none());
  m.def("comm_load", &comm_load);
  m.def("comm_unique_id", &comm_unique_id);
  m.def("comm_init", &comm_init);
  m.def("comm_destroy", &comm_destroy);
  m.def("comm_abort", &comm_abort);
  m.def("comm_async_error", &comm_async_error);
  m.def("comm_wait", &comm_wait);
  m.def("comm_allreduce", &comm_allreduce);
  m.def("comm_broadcast", &comm_broadcast);
  m.def("comm_allgather", &comm_allgather);
  m.def("gemm_attn_fwd", &gemm_attn_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("qkv"),
        py::arg("kbias"), py::arg("ctx"), py::arg("lse"), py::arg("B"), py::arg("S"), py::arg("H"), py::arg("seed"),
        py::arg("site"), py::arg("thr"), py::arg("dscale"), py::arg("cu"), py::arg("dmask"), py::arg("q_live"),
        py::arg("stats"), py::arg("cnt"), py::arg("err"), py::arg("xsite"), py::arg("cxc") = py::none(),
        py::arg("xc") = py::none(), py::arg("xres") = py::none(), py::arg("prefetch") = py::none(),
        py::arg("mode") = 1, py::arg("split") = -1);
  m.def("attn_fwd", &attn_fwd, py::arg("qkv"), py::arg("kbias"), py::arg("ctx"), py::arg("lse"), py::arg("B"),
        py::arg("S"), py::arg("H"), py::arg("seed"), py::arg("site"), py::arg("thr"), py::arg("dscale"), py::arg("cu"),
        py::arg("dmask"), py::arg("q_live") = 0, py::arg("cxc") = py::none(), py::arg("xc") = py::none(),
        py::arg("xres") = py::none(), py::arg("split") = -1);
  m.def("attn_bwd", &attn_bwd, py::arg("qkv"), py::arg("kbias"), py::arg("ctx"), py::arg("lse"), py::arg("dctx"),
        py::arg("delta"), py::arg("dqkv"), py::arg("B"), py::arg("S"), py::arg("H"), py::arg("seed"), py::arg("site"),
        py::arg("thr"), py::arg("dscale"), py::arg("cu"), py::arg("dmask"), py::arg("q_live") = 0,
        py::arg("dresc") = py::none(), py::arg("dres") = py::none(), py::arg("split") = -1);
  m.def("attn_bwd_proj", &attn_bwd_proj, py::arg("qkv"), py::arg("kbias"), py::arg("ctx"), py::arg("lse"),
        py::arg("dy"), py::arg("w"), py::arg("dqkv"), py::arg("B"), py::arg("S"), py::arg("H"), py::arg("seed"),
        py::arg("site"), py::arg("thr"), py::arg("dscale"), py::arg("cu"), py::arg("dmask"), py::arg("splits") = 1,
        py::arg("dresc") = py::none(), py::arg("dres") = py::none(), py::arg("split") = -1);
  m.def("mask_to_bias", &mask_to_bias);
  m.def("attn_set_split", [](int64_t on) { return (int64_t)fd_attn_set_split((int)on); });
  m.def("ln_fwd", &ln_fwd);
  m.def("ln_bwd", &ln_bwd);
  m.def("emb_fwd", &emb_fwd, py::arg("ids"), py::arg("word"), py::arg("pos"), py::arg("gamma"), py::arg("beta"),
        py::arg("y"), py::arg("mean"), py::arg("rstd"), py::arg("S"), py::arg("eps"), py::arg("seed"), py::arg("site"),
        py::arg("thr"), py::arg("dscale"), py::arg("row_map") = py::none(), py::arg("ln_epoch") = py::none(),
        py::arg("sorted") = py::none(), py::arg("perm") = py::none(), py::arg("ln_stats") = py::none());
  m.def("gemm_ln_set_diag", [](int64_t d) { fd_gemm_ln_set_diag((int)d); });
  m.def("gemm_dwb_set_mix", [](int64_t mode) { return (int64_t)fd_gemm_dwb_set_mix((int)mode); },
        "all-layer dW launch schedule: 0 plain, 1 mixed tiles when shorter (default), 2 forced; returns the old mode");
  m.def("gemm_dwb_mixed_launches", []() { return (int64_t)fd_gemm_dwb_mixed_launches(); });
  m.def("emb_bwd", &emb_bwd);
  m.def("colsum_bf16", &colsum_bf16);
  m.def("colsum_bf16_batched", &colsum_bf16_batched);
  m.def("colsum_batched", &colsum_batched);
  m.def("rank_sort", &rank_sort);
  m.def("head_fwd", &head_fwd, py::arg("hidden"), py::arg("B"), py::arg("S"), py::arg("W"), py::arg("bias"),
        py::arg("seed"), py::arg("site"), py::arg("thr"), py::arg("dscale"), py::arg("labels"), py::arg("logits"),
        py::arg("loss"), py::arg("dlogits"), py::arg("row_loss"), py::arg("cls"), py::arg("tlogits") = py::none(),
        py::arg("kd_T") = 1.0, py::arg("kd_alpha") = 1.0, py::arg("loss_acc") = py::none());
  m.def("head_bwd", &head_bwd, py::arg("hidden"), py::arg("B"), py::arg("S"), py::arg("W"), py::arg("seed"),
        py::arg("site"), py::arg("thr"), py::arg("dscale"), py::arg("dlogits"), py::arg("dW"), py::arg("db"),
        py::arg("dhidden"), py::arg("accumulate"), py::arg("cls") = py::none(), py::arg("gscale") = py::none(),
        py::arg("own") = py::none());
  m.def("head_ln_bwd", &head_ln_bwd);
  m.def("eval_metrics", &eval_metrics);
  m.def("adam", &adam);
  m.def("step_inc", &step_inc);
  m.def("scale_cast", &scale_cast);
  m.def("axpby", &axpby);
}
#endif  // FD_HOST_VALIDATION
