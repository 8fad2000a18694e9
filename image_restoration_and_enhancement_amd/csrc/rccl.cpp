// RCCL over xGMI behind the C ABI: the one collective of the data path, the broadcast of the frozen weight
// blobs from rank 0 (SURVEY.md §8b `irx_weights_bcast(handle, rcclComm)`, §8e).  The reference has no
// multi-device path at all (src/inference.py:52-57: one process, one device); this is build-side scope.
//
// librccl is resolved at first use with dlopen("librccl.so.1"): inside a PyTorch-ROCm process that soname is
// already mapped (torch's own RCCL), so the engine's communicator lives in the same RCCL instance as
// torch.distributed's; a plain C caller gets /opt/rocm's.  libirx.so itself keeps no link-time dependency on
// RCCL, so a single-GPU user never loads it.
#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <string>

#include <rccl/rccl.h>

#include "../../include/irx.h"
#include "irx_common.h"

namespace irx {
namespace {

struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
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

}  // namespace

// chunks of at most 1 GiB: the element count of one ncclBroadcast stays far inside every RCCL build's limits
void rccl_broadcast(void* comm, void* buf, size_t bytes, int root, hipStream_t s) {
  const RcclApi& a = need();
  IRX_CHECK(comm, "null communicator");
  IRX_CHECK(buf || bytes == 0, "null buffer");
  const size_t chunk = size_t(1) << 30;
  for (size_t off = 0; off < bytes; off += chunk) {
    const size_t n = bytes - off < chunk ? bytes - off : chunk;
    check(a.broadcast((char*)buf + off, (char*)buf + off, n, ncclUint8, root, (ncclComm_t)comm, s), "ncclBroadcast");
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
  IRX_CHECK(id && comm, "null argument");
  IRX_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / nranks");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  check(need().comm_init_rank(&c, nranks, u, rank), "ncclCommInitRank");
  *comm = c;
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
