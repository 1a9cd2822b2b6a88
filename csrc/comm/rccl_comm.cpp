// Native RCCL communicator for the FedAvg data path.
//
// The reference moves models with a hand-rolled TCP star: pickle + gzip, one
// 265 MB upload per client and one broadcast back (client1.py:276-336,
// server.py:29-114).  Here a round is one ncclAllReduce over the flat fp32
// parameter arena, issued on the caller's HIP stream so it orders with the
// fused scale/cast kernel that follows, over xGMI between the GPUs of a node.
//
// Rendezvous stays in torch.distributed (TCPStore): rank 0 creates the
// ncclUniqueId and the Python side broadcasts its 128 bytes; every rank then
// calls fd_comm_init.  The communicator is independent of torch's process
// group, so the framework's collectives do not depend on torch's NCCL wrapper
// (its watchdog, work objects, stream bookkeeping).
//
// Failure semantics (the reference bounds every socket with a 300 s timeout and retries,
// client1.py:22,280,323, server.py:10,92-112): a collective whose peer died never completes on
// its own.  fd_comm_wait polls the stream the collective was issued on together with
// ncclCommGetAsyncError, so the host learns of an RCCL-reported failure (a peer's broken
// connection) or of a timeout instead of blocking forever; the caller then aborts the
// communicator (fd_comm_abort = ncclCommAbort: it tears down the proxy threads and unblocks the
// kernels of the pending collective) and raises.
//
// RCCL itself is bound at run time (fd_comm_load): the process already holds
// the librccl that torch was built against, and linking a second copy from
// /opt/rocm would put two RCCL instances (two sets of proxy threads / IPC
// state) in one process.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

namespace {

thread_local std::string g_err;

struct Rccl {
  void* lib = nullptr;
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclBroadcast) Broadcast = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
  decltype(&ncclCommAbort) CommAbort = nullptr;
} R;

#define ncclGetUniqueId R.GetUniqueId
#define ncclCommInitRank R.CommInitRank
#define ncclCommDestroy R.CommDestroy
#define ncclAllReduce R.AllReduce
#define ncclBroadcast R.Broadcast
#define ncclAllGather R.AllGather
#define ncclGroupStart R.GroupStart
#define ncclGroupEnd R.GroupEnd
#define ncclGetErrorString R.GetErrorString
#define ncclCommGetAsyncError R.CommGetAsyncError
#define ncclCommAbort R.CommAbort

int fail(const char* what, ncclResult_t r) {
  g_err = std::string(what) + ": " + ncclGetErrorString(r);
  return (int)r == 0 ? 1 : (int)r;
}

ncclDataType_t dtype_of(int dtype) {
  switch (dtype) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat64;
    case 3: return ncclInt64;
    case 4: return ncclInt32;
    default: return ncclFloat32;
  }
}

}  // namespace

extern "C" {

const char* fd_comm_last_error() { return g_err.c_str(); }

// Bind the RCCL entry points from `path` (torch's librccl, already mapped).
int fd_comm_load(const char* path) {
  if (R.lib) return 0;
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    g_err = std::string("dlopen(") + path + "): " + dlerror();
    return 1;
  }
  auto sym = [&](const char* n) { return dlsym(h, n); };
  R.GetUniqueId = (decltype(R.GetUniqueId))sym("ncclGetUniqueId");
  R.CommInitRank = (decltype(R.CommInitRank))sym("ncclCommInitRank");
  R.CommDestroy = (decltype(R.CommDestroy))sym("ncclCommDestroy");
  R.AllReduce = (decltype(R.AllReduce))sym("ncclAllReduce");
  R.Broadcast = (decltype(R.Broadcast))sym("ncclBroadcast");
  R.AllGather = (decltype(R.AllGather))sym("ncclAllGather");
  R.GroupStart = (decltype(R.GroupStart))sym("ncclGroupStart");
  R.GroupEnd = (decltype(R.GroupEnd))sym("ncclGroupEnd");
  R.GetErrorString = (decltype(R.GetErrorString))sym("ncclGetErrorString");
  R.CommGetAsyncError = (decltype(R.CommGetAsyncError))sym("ncclCommGetAsyncError");
  R.CommAbort = (decltype(R.CommAbort))sym("ncclCommAbort");
  if (!R.GetUniqueId || !R.CommInitRank || !R.CommDestroy || !R.AllReduce || !R.Broadcast || !R.AllGather ||
      !R.GroupStart || !R.GroupEnd || !R.GetErrorString || !R.CommGetAsyncError || !R.CommAbort) {
    g_err = std::string("missing RCCL symbols in ") + path;
    R = Rccl{};
    return 2;
  }
  R.lib = h;
  return 0;
}

int fd_comm_loaded() { return R.lib != nullptr; }

int fd_comm_unique_id_bytes() { return (int)sizeof(ncclUniqueId); }

int fd_comm_get_unique_id(void* out) {
  if (!R.lib) { g_err = "RCCL not loaded (fd_comm_load)"; return 1; }
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return fail("ncclGetUniqueId", r);
  std::memcpy(out, &id, sizeof(id));
  return 0;
}

// The current HIP device must already be this rank's GPU.
int fd_comm_init(void** comm, int nranks, int rank, const void* id_bytes) {
  if (!R.lib) { g_err = "RCCL not loaded (fd_comm_load)"; return 1; }
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, sizeof(id));
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommInitRank(&c, nranks, id, rank);
  if (r != ncclSuccess) return fail("ncclCommInitRank", r);
  *comm = c;
  return 0;
}

// The communicator's asynchronous error state (ncclCommGetAsyncError): 0 = healthy,
// otherwise the ncclResult_t RCCL recorded (the message is left in fd_comm_last_error).
int fd_comm_async_error(void* comm) {
  if (!R.lib || !comm) { g_err = "communicator not initialised"; return 1; }
  ncclResult_t async = ncclSuccess;
  const ncclResult_t r = ncclCommGetAsyncError((ncclComm_t)comm, &async);
  if (r != ncclSuccess) return fail("ncclCommGetAsyncError", r);
  if (async != ncclSuccess && async != ncclInProgress) return fail("RCCL asynchronous error", async);
  return 0;
}

// Wait until everything issued on `st` (the collective last among it) has completed, checking the
// communicator's async error every poll.  Returns 0 when done, FD_COMM_TIMEOUT after timeout_ms,
// or the RCCL error code; a HIP error of the stream returns FD_COMM_HIP_ERROR.  Never aborts by
// itself: the caller decides (fd_comm_abort) -- the stream's pending work then stays queued.
#define FD_COMM_TIMEOUT 1001
#define FD_COMM_HIP_ERROR 1002
int fd_comm_wait(void* comm, hipStream_t st, long long timeout_ms) {
  const auto t0 = std::chrono::steady_clock::now();
  int sleep_us = 20;
  for (;;) {
    const hipError_t q = hipStreamQuery(st);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) {
      g_err = std::string("hipStreamQuery: ") + hipGetErrorString(q);
      return FD_COMM_HIP_ERROR;
    }
    const int a = fd_comm_async_error(comm);
    if (a) return a;
    const long long ms =
        std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_ms >= 0 && ms >= timeout_ms) {
      g_err = "collective did not complete within " + std::to_string(timeout_ms) + " ms (peer lost?)";
      return FD_COMM_TIMEOUT;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
    if (sleep_us < 2000) sleep_us *= 2;
  }
}

// ncclCommAbort: frees the communicator without the collective handshake of ncclCommDestroy
// (which would wait for the dead peer) and makes its pending kernels return.
int fd_comm_abort(void* comm) {
  if (!R.lib || !comm) return 0;
  const ncclResult_t r = ncclCommAbort((ncclComm_t)comm);
  return r == ncclSuccess ? 0 : fail("ncclCommAbort", r);
}

int fd_comm_destroy(void* comm) {
  if (!comm) return 0;
  const ncclResult_t r = ncclCommDestroy((ncclComm_t)comm);
  return r == ncclSuccess ? 0 : fail("ncclCommDestroy", r);
}

// op: 0 = sum, 1 = avg, 2 = max.  In place (send == recv) is allowed.
int fd_comm_allreduce(void* comm, const void* send, void* recv, long long count, int dtype, int op, hipStream_t st) {
  const ncclRedOp_t o = op == 1 ? ncclAvg : (op == 2 ? ncclMax : ncclSum);
  const ncclResult_t r = ncclAllReduce(send, recv, (size_t)count, dtype_of(dtype), o, (ncclComm_t)comm, st);
  return r == ncclSuccess ? 0 : fail("ncclAllReduce", r);
}

int fd_comm_broadcast(void* comm, void* buf, long long count, int dtype, int root, hipStream_t st) {
  const ncclResult_t r = ncclBroadcast(buf, buf, (size_t)count, dtype_of(dtype), root, (ncclComm_t)comm, st);
  return r == ncclSuccess ? 0 : fail("ncclBroadcast", r);
}

// recv holds nranks * count elements, rank-major.
int fd_comm_allgather(void* comm, const void* send, void* recv, long long count, int dtype, hipStream_t st) {
  const ncclResult_t r = ncclAllGather(send, recv, (size_t)count, dtype_of(dtype), (ncclComm_t)comm, st);
  return r == ncclSuccess ? 0 : fail("ncclAllGather", r);
}

// Bucketed all-reduce: `nb` in-place buffers reduced inside one group call (a
// single launch sequence; used for per-parameter-group averaging).
int fd_comm_allreduce_group(void* comm, void* const* bufs, const long long* counts, int nb, int dtype, int op,
                            hipStream_t st) {
  const ncclRedOp_t o = op == 1 ? ncclAvg : (op == 2 ? ncclMax : ncclSum);
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return fail("ncclGroupStart", r);
  for (int i = 0; i < nb; ++i) {
    r = ncclAllReduce(bufs[i], bufs[i], (size_t)counts[i], dtype_of(dtype), o, (ncclComm_t)comm, st);
    if (r != ncclSuccess) {
      ncclGroupEnd();
      return fail("ncclAllReduce(group)", r);
    }
  }
  r = ncclGroupEnd();
  return r == ncclSuccess ? 0 : fail("ncclGroupEnd", r);
}

}  // extern "C"
