// A communicator of our own over RCCL (xGMI between the GPUs of a node), issuing every collective
// on the caller's HIP stream.
//
// Why not only torch.distributed's ProcessGroupNCCL: it runs each collective on the process
// group's private stream, so a captured training step forks into that stream and joins back (a
// branch per collective in the HIP graph), and its watchdog thread polls events while we capture.
// Collectives enqueued on the step's own stream keep the captured graph a straight line (or on the
// encode side stream, which the step already forks for backward overlap), need no watchdog, and
// are ordered by the stream like any kernel.
//
// The library is the RCCL torch already loaded (same SONAME librccl.so.1, so one copy per
// process); its entry points are resolved with dlsym, no link-time dependency.  The unique id is
// distributed by the caller (ops/__init__.py via the process group's object broadcast).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"
#include "ewdml_ops.h"

namespace {

struct RcclApi {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclGetVersion) version = nullptr;
  std::string error;
};

template <typename F>
void rc_sym(void* h, const char* name, F& f, std::string& err) {
  f = reinterpret_cast<F>(dlsym(h, name));
  if (!f) err += std::string(" missing ") + name;
}

RcclApi& rc_api() {
  static RcclApi a;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // torch's copy, if loaded
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      a.error = std::string("cannot load librccl: ") + dlerror();
      return;
    }
    rc_sym(h, "ncclGetUniqueId", a.get_unique_id, a.error);
    rc_sym(h, "ncclCommInitRank", a.init_rank, a.error);
    rc_sym(h, "ncclCommDestroy", a.destroy, a.error);
    rc_sym(h, "ncclCommAbort", a.abort, a.error);
    rc_sym(h, "ncclAllGather", a.all_gather, a.error);
    rc_sym(h, "ncclAllReduce", a.all_reduce, a.error);
    rc_sym(h, "ncclReduceScatter", a.reduce_scatter, a.error);
    rc_sym(h, "ncclBroadcast", a.broadcast, a.error);
    rc_sym(h, "ncclSend", a.send, a.error);
    rc_sym(h, "ncclRecv", a.recv, a.error);
    rc_sym(h, "ncclGroupStart", a.group_start, a.error);
    rc_sym(h, "ncclGroupEnd", a.group_end, a.error);
    rc_sym(h, "ncclGetErrorString", a.error_string, a.error);
    rc_sym(h, "ncclGetVersion", a.version, a.error);
  });
  if (!a.error.empty()) throw std::runtime_error("ewdml rccl: " + a.error);
  return a;
}

void rc_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    RcclApi& a = rc_api();
    throw std::runtime_error(std::string("ewdml rccl: ") + what + " failed: " +
                             (a.error_string ? a.error_string(r) : "?"));
  }
}

ncclComm_t rc_comm(uintptr_t h) {
  if (!h) throw std::runtime_error("ewdml rccl: null communicator");
  return reinterpret_cast<ncclComm_t>(h);
}

ncclDataType_t rc_dtype(int code) {
  switch (code) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclUint8;
    case 4: return ncclInt32;
    case 5: return ncclFloat64;
    case 6: return ncclInt64;
    default: throw std::runtime_error("ewdml rccl: unknown dtype code");
  }
}

size_t rc_size(int code) {
  static const size_t sz[] = {4, 2, 2, 1, 4, 8, 8};
  return sz[code];
}

ncclRedOp_t rc_op(int code) {
  switch (code) {
    case 0: return ncclSum;
    case 1: return ncclMax;
    case 2: return ncclMin;
    case 3: return ncclAvg;
    default: throw std::runtime_error("ewdml rccl: unknown reduction");
  }
}

}  // namespace

std::string ew_rccl_unique_id() {
  ncclUniqueId id;
  rc_check(rc_api().get_unique_id(&id), "ncclGetUniqueId");
  return std::string(id.internal, sizeof(id.internal));
}

int ew_rccl_version() {
  int v = 0;
  rc_check(rc_api().version(&v), "ncclGetVersion");
  return v;
}

uintptr_t ew_rccl_init(const std::string& uid, int nranks, int rank, int device) {
  if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("ewdml rccl: bad unique id");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  EW_CHECK(hipSetDevice(device));
  ncclComm_t comm = nullptr;
  rc_check(rc_api().init_rank(&comm, nranks, id, rank), "ncclCommInitRank");
  return reinterpret_cast<uintptr_t>(comm);
}

void ew_rccl_destroy(uintptr_t h) {
  if (h) rc_check(rc_api().destroy(rc_comm(h)), "ncclCommDestroy");
}

void ew_rccl_all_gather(uintptr_t h, uintptr_t send, uintptr_t recv, long long count, int dtype,
                        uintptr_t stream) {
  rc_check(rc_api().all_gather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                               (size_t)count, rc_dtype(dtype), rc_comm(h), (hipStream_t)stream),
           "ncclAllGather");
}

void ew_rccl_all_reduce(uintptr_t h, uintptr_t send, uintptr_t recv, long long count, int dtype,
                        int op, uintptr_t stream) {
  rc_check(rc_api().all_reduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                               (size_t)count, rc_dtype(dtype), rc_op(op), rc_comm(h),
                               (hipStream_t)stream),
           "ncclAllReduce");
}

void ew_rccl_reduce_scatter(uintptr_t h, uintptr_t send, uintptr_t recv, long long count,
                            int dtype, int op, uintptr_t stream) {
  rc_check(rc_api().reduce_scatter(reinterpret_cast<const void*>(send),
                                   reinterpret_cast<void*>(recv), (size_t)count, rc_dtype(dtype),
                                   rc_op(op), rc_comm(h), (hipStream_t)stream),
           "ncclReduceScatter");
}

void ew_rccl_broadcast(uintptr_t h, uintptr_t send, uintptr_t recv, long long count, int dtype,
                       int root, uintptr_t stream) {
  rc_check(rc_api().broadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                              (size_t)count, rc_dtype(dtype), root, rc_comm(h),
                              (hipStream_t)stream),
           "ncclBroadcast");
}

// all-to-all of equal slices (count elements per peer) as one grouped send/recv round
void ew_rccl_all_to_all(uintptr_t h, uintptr_t send, uintptr_t recv, long long count, int dtype,
                        int nranks, uintptr_t stream) {
  RcclApi& a = rc_api();
  const ncclDataType_t dt = rc_dtype(dtype);
  const size_t bytes = (size_t)count * rc_size(dtype);
  rc_check(a.group_start(), "ncclGroupStart");
  for (int r = 0; r < nranks; ++r) {
    rc_check(a.send(reinterpret_cast<const char*>(send) + r * bytes, (size_t)count, dt, r,
                    rc_comm(h), (hipStream_t)stream),
             "ncclSend");
    rc_check(a.recv(reinterpret_cast<char*>(recv) + r * bytes, (size_t)count, dt, r, rc_comm(h),
                    (hipStream_t)stream),
             "ncclRecv");
  }
  rc_check(a.group_end(), "ncclGroupEnd");
}
