// comm.hip — single-process multi-device communicator (SURVEY.md §5 "Distributed comm
// backend": one process driving the node's GPUs, ncclCommInitAll; §8(b) tw_comm_init /
// tw_allgather_u64).
//
// The reference's N workers are a serial in-process loop (learning-experiment/compute_stats.py:
// 71-91, estimation-experiment/main.py:48-68), so its drop-in API runs in ONE process; the
// package spreads a call's blocks over the visible devices and combines their per-block
// integers here: an all-gather over RCCL (xGMI peer links), after which one device holds every
// block's count and the host copies them back once.
//
// RCCL is bound at run time (dlopen): the copy the host process already has loaded (PyTorch
// ships one) is preferred, so the process never holds two RCCL runtimes; otherwise the
// system's librccl.so.1 is loaded (TW_RCCL_LIB names another library: the tests' failure
// stub).  A process without RCCL gets TW_ERR_HIP from tw_comm_init and the Python layer
// gathers on the host instead — the same integers either way.
//
// Failure detection: a collective whose peer fails never completes, so the
// caller that needs its result waits through tw_comm_wait — bounded, polling
// ncclCommGetAsyncError on every device's communicator and the streams' progress; an RCCL
// error or the deadline aborts the communicator (ncclCommAbort, so its kernels stop holding
// the GPUs) and returns TW_ERR_HIP; the handle is then dead and later calls on it fail at once.
#include "tw_common.h"
#include <chrono>
#include <cstdlib>
#include <dlfcn.h>
#include <mutex>
#include <thread>
#include <vector>

namespace tw {

typedef struct ncclComm* ncclComm_t;
typedef int ncclResult_t;  // 0 = ncclSuccess
constexpr int kNcclUint64 = 5;
constexpr int kNcclFloat64 = 8;
constexpr ncclResult_t kNcclInProgress = 7;

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*initAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*allGather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*groupStart)() = nullptr;
  ncclResult_t (*groupEnd)() = nullptr;
  const char* (*errStr)(ncclResult_t) = nullptr;
  ncclResult_t (*asyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*abort)(ncclComm_t) = nullptr;
};

static Rccl g_rccl;
static std::mutex g_mu;
static std::vector<std::vector<ncclComm_t>> g_comms;  // handle -> one comm per device
static std::vector<std::vector<int>> g_devs;          // handle -> its devices
static std::vector<std::vector<hipEvent_t>> g_pre;    // handle -> per device, recorded on the
                                                      // stream just before the collective
static std::vector<char> g_dead;                      // handle -> aborted after a failure
static int64_t g_wait_ms = 60000;                     // tw_comm_set_timeout
// the work queued on a stream BEFORE the collective gets its own, generous deadline
// (tw_comm_set_prior_timeout): a legitimately long count must not be taken for an RCCL failure,
// but a wedged stream (an earlier collective that never completes, a hung kernel) must still
// end in an error rather than an unbounded wait
static int64_t g_prior_ms = 600000;

static bool load_rccl() {
  if (g_rccl.h) return true;
  // an RCCL already in the process first (by soname or by the name PyTorch linked), then the
  // system one
  const char* names[] = {"librccl.so.1", "librccl.so"};
  void* h = nullptr;
  const char* over = std::getenv("TW_RCCL_LIB");
  if (over && *over) {
    h = dlopen(over, RTLD_NOW | RTLD_LOCAL);
  } else {
    for (const char* n : names)
      if ((h = dlopen(n, RTLD_NOW | RTLD_NOLOAD)) != nullptr) break;
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  }
  if (!h) return false;
  Rccl r;
  r.h = h;
  r.initAll = (decltype(r.initAll))dlsym(h, "ncclCommInitAll");
  r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
  r.allGather = (decltype(r.allGather))dlsym(h, "ncclAllGather");
  r.groupStart = (decltype(r.groupStart))dlsym(h, "ncclGroupStart");
  r.groupEnd = (decltype(r.groupEnd))dlsym(h, "ncclGroupEnd");
  r.errStr = (decltype(r.errStr))dlsym(h, "ncclGetErrorString");
  r.asyncError = (decltype(r.asyncError))dlsym(h, "ncclCommGetAsyncError");
  r.abort = (decltype(r.abort))dlsym(h, "ncclCommAbort");
  if (!r.initAll || !r.destroy || !r.allGather || !r.groupStart || !r.groupEnd ||
      !r.asyncError || !r.abort)
    return false;
  g_rccl = r;
  return true;
}

static const char* nccl_err(ncclResult_t e) {
  return g_rccl.errStr ? g_rccl.errStr(e) : "RCCL error";
}

// An event per device recorded on the collective's stream right before it is enqueued:
// tw_comm_wait's deadline starts only once the work queued before the collective (a count of
// any length) has drained, so a slow count is never taken for an RCCL failure.  Without a
// device (the CPU test's stub) no event exists and the deadline covers the whole stream.
static void mark_pre(int32_t comm, void* const* streams) {
  std::lock_guard<std::mutex> lk(g_mu);
  std::vector<hipEvent_t>& pre = g_pre[comm];
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) cur = -1;
  for (size_t k = 0; k < pre.size(); ++k) {
    if (hipSetDevice(g_devs[comm][k]) != hipSuccess) continue;
    if (!pre[k] && hipEventCreateWithFlags(&pre[k], hipEventDisableTiming) != hipSuccess)
      pre[k] = nullptr;
    if (pre[k] && hipEventRecord(pre[k], (hipStream_t)streams[k]) != hipSuccess) {
      (void)hipEventDestroy(pre[k]);
      pre[k] = nullptr;
    }
  }
  if (cur >= 0) (void)hipSetDevice(cur);
  (void)hipGetLastError();  // no sticky error from a device-less process
}

static int allgather(int32_t comm, const void* const* send, void* const* recv, int64_t count,
                     int dtype, void* const* streams) {
  std::vector<ncclComm_t> cs;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    TW_ARG_CHECK(comm >= 0 && comm < (int32_t)g_comms.size() && !g_comms[comm].empty(),
                 "tw_allgather: unknown communicator %d", comm);
    if (g_dead[comm]) {
      set_error("tw_allgather: communicator %d was aborted after an RCCL failure", comm);
      return TW_ERR_HIP;
    }
    cs = g_comms[comm];
  }
  TW_ARG_CHECK(count >= 0 && send && recv && streams, "tw_allgather: bad arguments");
  if (count == 0) return TW_OK;
  mark_pre(comm, streams);
  ncclResult_t e = g_rccl.groupStart();
  for (size_t k = 0; k < cs.size() && e == 0; ++k)
    e = g_rccl.allGather(send[k], recv[k], (size_t)count, dtype, cs[k], (hipStream_t)streams[k]);
  const ncclResult_t e2 = g_rccl.groupEnd();
  if (e == 0) e = e2;
  if (e != 0) {
    set_error("tw_allgather: %s", nccl_err(e));
    return TW_ERR_HIP;
  }
  return TW_OK;
}

// abort every device's communicator of a handle (caller holds g_mu)
static void abort_comm(int32_t comm) {
  for (ncclComm_t c : g_comms[comm]) g_rccl.abort(c);
  g_dead[comm] = 1;
}

static int wait_comm(int32_t comm, void* const* streams, int64_t timeout_ms) {
  std::vector<ncclComm_t> cs;
  std::vector<hipEvent_t> pre;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    TW_ARG_CHECK(comm >= 0 && comm < (int32_t)g_comms.size() && !g_comms[comm].empty(),
                 "tw_comm_wait: unknown communicator %d", comm);
    if (g_dead[comm]) {
      set_error("tw_comm_wait: communicator %d was aborted after an RCCL failure", comm);
      return TW_ERR_HIP;
    }
    cs = g_comms[comm];
    pre = g_pre[comm];
  }
  TW_ARG_CHECK(streams != nullptr, "tw_comm_wait: streams");
  const int64_t limit = timeout_ms > 0 ? timeout_ms : g_wait_ms;
  auto fail = [&](const char* what, const char* detail) {
    std::lock_guard<std::mutex> lk(g_mu);
    abort_comm(comm);
    set_error("tw_comm_wait: %s (%s); communicator %d aborted", what, detail, comm);
    return TW_ERR_HIP;
  };
  // an RCCL error on any device's communicator (a peer that failed, a broken link)
  auto async_error = [&]() -> int {
    for (ncclComm_t c : cs) {
      ncclResult_t ae = 0;
      const ncclResult_t e = g_rccl.asyncError(c, &ae);
      if (e != 0) return fail("ncclCommGetAsyncError failed", nccl_err(e));
      if (ae != 0 && ae != kNcclInProgress) return fail("RCCL asynchronous error", nccl_err(ae));
    }
    return TW_OK;
  };
  // first the work queued before the collective, under its own deadline
  const auto tp = std::chrono::steady_clock::now();
  for (bool before = true; before;) {
    if (const int rc = async_error()) return rc;
    before = false;
    for (hipEvent_t ev : pre) {
      if (!ev) continue;
      const hipError_t q = hipEventQuery(ev);
      if (q == hipErrorNotReady) {
        before = true;
      } else if (q != hipSuccess) {
        return fail("event query failed", hipGetErrorString(q));
      }
    }
    if (!before) break;
    const int64_t ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                           std::chrono::steady_clock::now() - tp).count();
    if (ms > g_prior_ms)
      return fail("the work queued before the collective did not finish in time",
                  "prior deadline");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  const auto t0 = std::chrono::steady_clock::now();  // the collective's own deadline
  for (;;) {
    if (const int rc = async_error()) return rc;
    bool done = true;
    for (size_t k = 0; k < cs.size(); ++k) {
      const hipError_t q = hipStreamQuery((hipStream_t)streams[k]);
      if (q == hipErrorNotReady) {
        done = false;
      } else if (q != hipSuccess) {
        return fail("stream query failed", hipGetErrorString(q));
      }
    }
    if (done) return TW_OK;
    const int64_t ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                           std::chrono::steady_clock::now() - t0).count();
    if (ms > limit) return fail("collective did not complete in time", "deadline");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

}  // namespace tw

using namespace tw;

extern "C" int tw_comm_init(int32_t ndev, const int32_t* devs, int32_t* out_comm) {
  TW_ARG_CHECK(ndev >= 1 && ndev <= 64 && devs && out_comm, "tw_comm_init: 1..64 devices");
  for (int i = 0; i < ndev; ++i)
    for (int j = 0; j < i; ++j)
      TW_ARG_CHECK(devs[i] != devs[j], "tw_comm_init: device %d listed twice", devs[i]);
  std::lock_guard<std::mutex> lk(g_mu);
  if (!load_rccl()) {
    set_error("tw_comm_init: RCCL (librccl.so.1) is not available");
    return TW_ERR_HIP;
  }
  std::vector<int> dl(devs, devs + ndev);
  std::vector<ncclComm_t> cs(ndev);
  const ncclResult_t e = g_rccl.initAll(cs.data(), ndev, dl.data());
  if (e != 0) {
    set_error("tw_comm_init: ncclCommInitAll: %s", nccl_err(e));
    return TW_ERR_HIP;
  }
  g_comms.push_back(cs);
  g_devs.push_back(dl);
  g_pre.push_back(std::vector<hipEvent_t>(ndev, nullptr));
  g_dead.push_back(0);
  *out_comm = (int32_t)g_comms.size() - 1;
  return TW_OK;
}

extern "C" int tw_comm_destroy(int32_t comm) {
  std::lock_guard<std::mutex> lk(g_mu);
  TW_ARG_CHECK(comm >= 0 && comm < (int32_t)g_comms.size() && !g_comms[comm].empty(),
               "tw_comm_destroy: unknown communicator %d", comm);
  if (!g_dead[comm])
    for (ncclComm_t c : g_comms[comm]) g_rccl.destroy(c);
  g_comms[comm].clear();
  for (hipEvent_t& ev : g_pre[comm])
    if (ev) {
      (void)hipEventDestroy(ev);
      ev = nullptr;
    }
  return TW_OK;
}

extern "C" int tw_comm_wait(int32_t comm, void* const* streams, int64_t timeout_ms) {
  return wait_comm(comm, streams, timeout_ms);
}

extern "C" int tw_comm_set_timeout(int64_t ms) {
  TW_ARG_CHECK(ms > 0, "tw_comm_set_timeout: ms > 0");
  g_wait_ms = ms;
  return TW_OK;
}

extern "C" int tw_comm_set_prior_timeout(int64_t ms) {
  TW_ARG_CHECK(ms > 0, "tw_comm_set_prior_timeout: ms > 0");
  g_prior_ms = ms;
  return TW_OK;
}

extern "C" int tw_allgather_u64(int32_t comm, const uint64_t* const* d_send,
                                uint64_t* const* d_recv, int64_t count, void* const* streams) {
  return allgather(comm, (const void* const*)d_send, (void* const*)d_recv, count, kNcclUint64,
                   streams);
}

extern "C" int tw_allgather_f64(int32_t comm, const double* const* d_send, double* const* d_recv,
                                int64_t count, void* const* streams) {
  return allgather(comm, (const void* const*)d_send, (void* const*)d_recv, count, kNcclFloat64,
                   streams);
}
