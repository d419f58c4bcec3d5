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

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
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

void ew_rccl_abort(uintptr_t h) {
  if (h) rc_check(rc_api().abort(rc_comm(h)), "ncclCommAbort");
}

// ---------------------------------------------------------------------------------------------
// Step watchdog.  The data-plane collectives run on the step's own stream (no process-group
// watchdog sees them), so a stalled peer would hang the surviving ranks inside a graph replay or a
// synchronize.  After each step the host enqueues a one-thread kernel that writes the step's
// sequence number into host-pinned memory (ew_rccl_watch); a thread compares it with the issued
// sequence and, once a step has been outstanding for longer than the timeout, releases the test
// spin flags, aborts the communicator (RCCL kernels waiting on a peer return) from a helper thread,
// waits a bounded moment for the stream to drain, and ends the process with a non-zero exit code.
// The watchdog thread makes no HIP call while it watches: a thread blocked in a device
// synchronize can hold the runtime's locks, and an hipEventQuery would wait behind it.  No exec,
// no retry: the launcher sees the failure (the reference's straggler kill intent,
// src/distributed_nn.py:50-59, src/model_ops/lenet.py:188-255).
// ---------------------------------------------------------------------------------------------
namespace {

__global__ void k_watch_mark(unsigned long long* done, unsigned long long seq) {
  __hip_atomic_store(done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Watchdog {
  ncclComm_t comm = nullptr;
  double timeout_s = 600.0;
  int exit_code = 3;
  unsigned long long* done = nullptr;  // host-pinned, written by k_watch_mark
  unsigned long long issued = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<unsigned long long, std::chrono::steady_clock::time_point>> pending;
  std::vector<volatile int*> release;  // host flags set to 1 on abort (test spin kernels)
  bool stop = false;
  std::thread th;

  unsigned long long completed() const {
    return __atomic_load_n(done, __ATOMIC_ACQUIRE);
  }

  [[noreturn]] void fire(double waited) {
    std::fprintf(stderr,
                 "ewdml watchdog: a step's collectives did not complete after %.1f s (timeout "
                 "%.1f s); aborting the RCCL communicator and exiting with code %d\n",
                 waited, timeout_s, exit_code);
    std::fflush(stderr);
    for (volatile int* f : release) *f = 1;
    std::atomic<bool> aborted{false};
    if (comm) {  // ncclCommAbort may block on the runtime: bounded wait, then exit regardless
      ncclComm_t c = comm;
      std::thread([c, &aborted] {
        rc_api().abort(c);
        aborted = true;
      }).detach();
    }
    const unsigned long long want = pending.empty() ? 0 : pending.front().first;
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::steady_clock::now() - t0 < std::chrono::seconds(4) &&
           !(aborted.load() && completed() >= want))
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    std::_Exit(exit_code);
  }

  void loop() {
    std::unique_lock<std::mutex> lk(mu);
    while (!stop) {
      cv.wait_for(lk, std::chrono::milliseconds(50));
      const unsigned long long c = completed();
      while (!pending.empty() && pending.front().first <= c) pending.pop_front();
      if (!pending.empty()) {
        const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() -
                                                            pending.front().second).count();
        if (waited > timeout_s) fire(waited);
      }
    }
  }
};

Watchdog* wd_of(uintptr_t h) {
  if (!h) throw std::runtime_error("ewdml watchdog: null handle");
  return reinterpret_cast<Watchdog*>(h);
}

__global__ void k_test_spin(const int* flag, unsigned long long max_ticks) {
  // test-only stall: waits for a host-pinned flag, bounded by max_ticks of the 100 MHz constant
  // clock so the grid always drains on its own
  const unsigned long long t0 = wall_clock64();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 &&
         wall_clock64() - t0 < max_ticks)
    __builtin_amdgcn_s_sleep(64);
}

}  // namespace

uintptr_t ew_rccl_watchdog_start(uintptr_t comm, int device, double timeout_s, int exit_code) {
  auto* w = new Watchdog();
  w->comm = comm ? rc_comm(comm) : nullptr;
  if (comm) rc_api();  // resolve ncclCommAbort now, not inside fire()
  EW_CHECK(hipSetDevice(device));
  void* p = nullptr;
  EW_CHECK(hipHostMalloc(&p, 64, hipHostMallocCoherent));
  std::memset(p, 0, 64);
  w->done = reinterpret_cast<unsigned long long*>(p);
  w->timeout_s = timeout_s;
  w->exit_code = exit_code;
  w->th = std::thread([w] { w->loop(); });
  return reinterpret_cast<uintptr_t>(w);
}

void ew_rccl_watch(uintptr_t h, uintptr_t stream) {
  Watchdog* w = wd_of(h);
  unsigned long long seq;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    seq = ++w->issued;
    w->pending.emplace_back(seq, std::chrono::steady_clock::now());
  }
  hipLaunchKernelGGL(k_watch_mark, dim3(1), dim3(1), 0, (hipStream_t)stream, w->done, seq);
  EW_CHECK_LAUNCH();
}

int ew_rccl_watch_pending(uintptr_t h) {
  Watchdog* w = wd_of(h);
  std::lock_guard<std::mutex> lk(w->mu);
  const unsigned long long c = w->completed();
  int n = 0;
  for (auto& p : w->pending) n += p.first > c;
  return n;
}

void ew_rccl_watchdog_stop(uintptr_t h) {
  Watchdog* w = wd_of(h);
  {
    std::lock_guard<std::mutex> lk(w->mu);
    w->stop = true;
  }
  w->cv.notify_all();
  if (w->th.joinable()) w->th.join();
  (void)hipHostFree(w->done);
  delete w;
}

// test hooks: a host-pinned flag released by the watchdog on abort, and a kernel stalling a
// stream on it (bounded)
uintptr_t ew_test_flag_alloc() {
  void* p = nullptr;
  EW_CHECK(hipHostMalloc(&p, 64, hipHostMallocCoherent));
  std::memset(p, 0, 64);
  return reinterpret_cast<uintptr_t>(p);
}
void ew_test_flag_free(uintptr_t f) {
  if (f) EW_CHECK(hipHostFree(reinterpret_cast<void*>(f)));
}
void ew_watchdog_release_flag(uintptr_t h, uintptr_t f) {
  Watchdog* w = wd_of(h);
  std::lock_guard<std::mutex> lk(w->mu);
  w->release.push_back(reinterpret_cast<volatile int*>(f));
}
void ew_test_spin(uintptr_t flag, double max_s, uintptr_t stream) {
  hipLaunchKernelGGL(k_test_spin, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     reinterpret_cast<const int*>(flag), (unsigned long long)(max_s * 1e8));
  EW_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------------------------
// Shape of a captured HIP graph (node count per type, edges, forks / joins): whether a step graph
// is a straight line, which ROCm replays with one batched submission, or a DAG, which it walks
// node by node from the host.  `dot_path`: also hipGraphDebugDotPrint.
// ---------------------------------------------------------------------------------------------
std::vector<long long> ew_graph_info(uintptr_t graph, const std::string& dot_path) {
  hipGraph_t g = reinterpret_cast<hipGraph_t>(graph);
  if (!g) throw std::runtime_error("ewdml graph_info: null graph");
  size_t n = 0, ne = 0;
  EW_CHECK(hipGraphGetNodes(g, nullptr, &n));
  std::vector<hipGraphNode_t> nodes(n);
  if (n) EW_CHECK(hipGraphGetNodes(g, nodes.data(), &n));
  EW_CHECK(hipGraphGetEdges(g, nullptr, nullptr, &ne));
  std::vector<hipGraphNode_t> from(ne), to(ne);
  if (ne) EW_CHECK(hipGraphGetEdges(g, from.data(), to.data(), &ne));
  // out: [nodes, edges, forks (out-degree > 1), joins (in-degree > 1), roots, then count per
  // hipGraphNodeType 0..15]
  std::vector<long long> out(5 + 16, 0);
  out[0] = (long long)n;
  out[1] = (long long)ne;
  for (size_t i = 0; i < n; ++i) {
    hipGraphNodeType t;
    EW_CHECK(hipGraphNodeGetType(nodes[i], &t));
    if ((int)t >= 0 && (int)t < 16) out[5 + (int)t] += 1;
    size_t od = 0, id = 0;
    EW_CHECK(hipGraphNodeGetDependentNodes(nodes[i], nullptr, &od));
    EW_CHECK(hipGraphNodeGetDependencies(nodes[i], nullptr, &id));
    out[2] += od > 1;
    out[3] += id > 1;
    out[4] += id == 0;
  }
  if (!dot_path.empty()) EW_CHECK(hipGraphDebugDotPrint(g, dot_path.c_str(), 0));
  return out;
}
