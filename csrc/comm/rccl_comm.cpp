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
// RCCL itself is bound at run time (fd_comm_load): the process already holds
// the librccl that torch was built against, and linking a second copy from
// /opt/rocm would put two RCCL instances (two sets of proxy threads / IPC
// state) in one process.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <string>

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
  if (!R.GetUniqueId || !R.CommInitRank || !R.CommDestroy || !R.AllReduce || !R.Broadcast || !R.AllGather ||
      !R.GroupStart || !R.GroupEnd || !R.GetErrorString) {
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
