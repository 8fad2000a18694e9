// RCCL over xGMI behind the C ABI: the one collective of the data path, the broadcast of the frozen weight
// blobs from rank 0 (SURVEY.md §8b `irx_weights_bcast(handle, rcclComm)`, §8e).  The reference has no
// multi-device path at all (src/inference.py:52-57: one process, one device); this is build-side scope.
//
// librccl is resolved at first use with dlopen("librccl.so.1"): inside a PyTorch-ROCm process that soname is
// already mapped (torch's own RCCL), so the engine's communicator lives in the same RCCL instance as
// torch.distributed's; a plain C caller gets /opt/rocm's.  libirx.so itself keeps no link-time dependency on
// RCCL, so a single-GPU user never loads it.
#include <dlfcn.h>

#include <chrono>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>

#include <rccl/rccl.h>

#include "../../include/irx.h"
#include "irx_common.h"

namespace irx {
namespace {

struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_init_rank_config)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
  ncclResult_t (*comm_get_async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  std::string load_error;
  bool ok = false;
};

const RcclApi& api() {
  static RcclApi a;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      a.load_error = std::string("cannot load librccl: ") + (e ? e : "?");
      return;
    }
    auto sym = [&](const char* n) {
      void* p = dlsym(h, n);
      if (!p && a.load_error.empty()) a.load_error = std::string("librccl lacks ") + n;
      return p;
    };
    a.get_unique_id = (decltype(a.get_unique_id))sym("ncclGetUniqueId");
    a.comm_init_rank = (decltype(a.comm_init_rank))sym("ncclCommInitRank");
    a.comm_init_rank_config = (decltype(a.comm_init_rank_config))sym("ncclCommInitRankConfig");
    a.comm_get_async_error = (decltype(a.comm_get_async_error))sym("ncclCommGetAsyncError");
    a.comm_abort = (decltype(a.comm_abort))sym("ncclCommAbort");
    a.comm_destroy = (decltype(a.comm_destroy))sym("ncclCommDestroy");
    a.broadcast = (decltype(a.broadcast))sym("ncclBroadcast");
    a.error_string = (decltype(a.error_string))sym("ncclGetErrorString");
    a.ok = a.load_error.empty();
  });
  return a;
}

const RcclApi& need() {
  const RcclApi& a = api();
  IRX_CHECK(a.ok, a.load_error);
  return a;
}

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw Error(std::string(what) + ": " + need().error_string(r));
}

// A communicator made with blocking = 0 may answer ncclInProgress to any call: its work then finishes on RCCL's own
// threads and ncclCommGetAsyncError reports when.  Polls until it leaves ncclInProgress or `deadline` passes.
ncclResult_t wait_async(ncclComm_t c, std::chrono::steady_clock::time_point deadline, bool* timed_out) {
  const RcclApi& a = need();
  *timed_out = false;
  for (;;) {
    ncclResult_t st = ncclInProgress;
    const ncclResult_t r = a.comm_get_async_error(c, &st);
    if (r != ncclSuccess) return r;
    if (st != ncclInProgress) return st;
    if (std::chrono::steady_clock::now() >= deadline) {
      *timed_out = true;
      return ncclInProgress;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
}

// Enqueue-side waits of a broadcast on a non-blocking communicator (the GPU work itself is ordered on the stream).
constexpr int kEnqueueTimeoutMs = 300000;

}  // namespace

// Communicator init with a deadline.  timeout_ms <= 0: the blocking ncclCommInitRank.  Otherwise
// ncclCommInitRankConfig with blocking = 0, polled with ncclCommGetAsyncError; on an error or at the deadline the
// half-made communicator is released with ncclCommAbort and an error is raised, so a rank whose peers never arrive
// (or fail partway) leaves the init instead of blocking inside it.
void* rccl_comm_init(const unsigned char* id, int nranks, int rank, int timeout_ms) {
  const RcclApi& a = need();
  IRX_CHECK(id, "null argument");
  IRX_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / nranks");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  if (timeout_ms <= 0) {
    check(a.comm_init_rank(&c, nranks, u, rank), "ncclCommInitRank");
    return c;
  }
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t r = a.comm_init_rank_config(&c, nranks, u, rank, &cfg);
  bool timed_out = false;
  if (r == ncclInProgress || (r == ncclSuccess && c)) r = wait_async(c, deadline, &timed_out);
  if (r == ncclSuccess) return c;
  if (c) a.comm_abort(c);
  if (timed_out)
    throw Error("ncclCommInitRankConfig: rank " + std::to_string(rank) + " of " + std::to_string(nranks) +
                " did not finish within " + std::to_string(timeout_ms) + " ms (communicator aborted)");
  throw Error(std::string("ncclCommInitRankConfig: ") + a.error_string(r) + " (communicator aborted)");
}

// chunks of at most 1 GiB: the element count of one ncclBroadcast stays far inside every RCCL build's limits
void rccl_broadcast(void* comm, void* buf, size_t bytes, int root, hipStream_t s) {
  const RcclApi& a = need();
  IRX_CHECK(comm, "null communicator");
  IRX_CHECK(buf || bytes == 0, "null buffer");
  const size_t chunk = size_t(1) << 30;
  for (size_t off = 0; off < bytes; off += chunk) {
    const size_t n = bytes - off < chunk ? bytes - off : chunk;
    ncclResult_t r = a.broadcast((char*)buf + off, (char*)buf + off, n, ncclUint8, root, (ncclComm_t)comm, s);
    if (r == ncclInProgress) {   // (a non-blocking communicator: wait for the enqueue before the next chunk)
      bool timed_out = false;
      r = wait_async((ncclComm_t)comm,
                     std::chrono::steady_clock::now() + std::chrono::milliseconds(kEnqueueTimeoutMs), &timed_out);
      IRX_CHECK(!timed_out, "ncclBroadcast: enqueue did not finish");
    }
    check(r, "ncclBroadcast");
  }
}

}  // namespace irx

using namespace irx;

#define RCCL_API_BEGIN try {
#define RCCL_API_END                 \
  return 0;                          \
  }                                  \
  catch (const std::exception& e) {  \
    set_error(e.what());             \
    return -1;                       \
  }                                  \
  catch (...) {                      \
    set_error("unknown error");      \
    return -1;                       \
  }

extern "C" {

int irx_rccl_available(void) { return api().ok ? 1 : 0; }

int irx_rccl_unique_id(unsigned char* id) {
  RCCL_API_BEGIN
  IRX_CHECK(id, "null argument");
  static_assert(sizeof(ncclUniqueId) == IRX_RCCL_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  check(need().get_unique_id(&u), "ncclGetUniqueId");
  std::memcpy(id, &u, sizeof(u));
  RCCL_API_END
}

int irx_rccl_comm_init(const unsigned char* id, int nranks, int rank, void** comm) {
  RCCL_API_BEGIN
  IRX_CHECK(comm, "null argument");
  *comm = rccl_comm_init(id, nranks, rank, 0);
  RCCL_API_END
}

int irx_rccl_comm_init_timeout(const unsigned char* id, int nranks, int rank, int timeout_ms, void** comm) {
  RCCL_API_BEGIN
  IRX_CHECK(comm, "null argument");
  *comm = nullptr;
  *comm = rccl_comm_init(id, nranks, rank, timeout_ms);
  RCCL_API_END
}

int irx_rccl_comm_destroy(void* comm) {
  RCCL_API_BEGIN
  if (comm) check(need().comm_destroy((ncclComm_t)comm), "ncclCommDestroy");
  RCCL_API_END
}

int irx_rccl_broadcast(void* comm, void* buf, size_t bytes, int root, void* stream) {
  RCCL_API_BEGIN
  rccl_broadcast(comm, buf, bytes, root, (hipStream_t)stream);
  RCCL_API_END
}

}  // extern "C"
