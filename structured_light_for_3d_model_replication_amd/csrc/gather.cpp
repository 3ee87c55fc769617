// gather.cpp — the final point-cloud gather of a view-sharded scan over RCCL (xGMI).
//
// SURVEY §8(e) / north star: turntable views are sharded view-per-GPU; the ONLY collective of
// the path is the gather of the finished clouds to one rank at the end of the job (the
// reference has no collective at all: its batch loop is serial, server/processing.py:314-334).
// Exact-size gatherv: every rank's counts travel by one ncclAllGather of int64, then one
// ncclGroupStart/End of point-to-point ncclSend / ncclRecv moves exactly the bytes each rank
// holds (no padding to the largest rank) -- on a fully connected xGMI mesh the root receives
// from all peers at once, one link each.
//
// RCCL is resolved at run time (dlopen, RTLD_NOLOAD first): the process normally already has
// the librccl.so.1 that torch loaded, and a communicator made here must live in that same
// library instance as torch's process group.  libslgpu.so itself does not depend on RCCL.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/slgpu.h"

int slg_internal_fail(int code, const char* fmt, ...);   // slgpu.hip: sets slg_last_error()

namespace {

struct RcclApi {
  void* handle = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

RcclApi* rccl() {
  static RcclApi api;
  static bool tried = false;
  if (tried) return api.handle ? &api : nullptr;
  tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);   // the one torch already loaded
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
  if (!h) h = dlopen("librccl.so", RTLD_NOW);
  if (!h) return nullptr;
#define SLG_SYM(field, name) api.field = reinterpret_cast<decltype(api.field)>(dlsym(h, name)); if (!api.field) return nullptr;
  SLG_SYM(get_unique_id, "ncclGetUniqueId")
  SLG_SYM(comm_init_rank, "ncclCommInitRank")
  SLG_SYM(comm_destroy, "ncclCommDestroy")
  SLG_SYM(all_gather, "ncclAllGather")
  SLG_SYM(send, "ncclSend")
  SLG_SYM(recv, "ncclRecv")
  SLG_SYM(group_start, "ncclGroupStart")
  SLG_SYM(group_end, "ncclGroupEnd")
  SLG_SYM(error_string, "ncclGetErrorString")
#undef SLG_SYM
  api.handle = h;
  return &api;
}

int nccl_fail(RcclApi* a, ncclResult_t r, const char* what) {
  return slg_internal_fail(SLG_ERR_HIP, "%s: %s", what, a->error_string(r));
}

}  // namespace

struct slg_gather_comm {
  ncclComm_t comm;
  int32_t n_ranks;
  int32_t rank;
};

extern "C" {

int32_t slg_gather_unique_id(uint8_t* id) {
  if (!id) return slg_internal_fail(SLG_ERR_INVALID, "id NULL");
  RcclApi* a = rccl();
  if (!a) return slg_internal_fail(SLG_ERR_UNSUPPORTED, "RCCL (librccl.so.1) not found");
  static_assert(sizeof(ncclUniqueId) == SLG_GATHER_ID_BYTES, "unique id size");
  ncclUniqueId u;
  const ncclResult_t r = a->get_unique_id(&u);
  if (r != ncclSuccess) return nccl_fail(a, r, "ncclGetUniqueId");
  memcpy(id, &u, sizeof(u));
  return SLG_OK;
}

int32_t slg_gather_init(slg_gather_comm** out, int32_t n_ranks, int32_t rank, const uint8_t* id) {
  if (!out || !id || n_ranks < 1 || rank < 0 || rank >= n_ranks)
    return slg_internal_fail(SLG_ERR_INVALID, "bad gather init argument");
  RcclApi* a = rccl();
  if (!a) return slg_internal_fail(SLG_ERR_UNSUPPORTED, "RCCL (librccl.so.1) not found");
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c;
  const ncclResult_t r = a->comm_init_rank(&c, n_ranks, u, rank);   // on the current HIP device
  if (r != ncclSuccess) return nccl_fail(a, r, "ncclCommInitRank");
  *out = new slg_gather_comm{c, n_ranks, rank};
  return SLG_OK;
}

int32_t slg_gather_counts(slg_gather_comm* g, const int64_t* counts, int32_t n_per_rank, int64_t* all_counts,
                          void* stream) {
  if (!g || !counts || !all_counts || n_per_rank < 1) return slg_internal_fail(SLG_ERR_INVALID, "bad argument");
  RcclApi* a = rccl();
  const ncclResult_t r = a->all_gather(counts, all_counts, size_t(n_per_rank), ncclInt64, g->comm,
                                       static_cast<hipStream_t>(stream));
  if (r != ncclSuccess) return nccl_fail(a, r, "ncclAllGather");
  return SLG_OK;
}

int32_t slg_gatherv_plan(int32_t n_ranks, int32_t rank, int32_t root, int64_t send_bytes, const int64_t* recv_bytes,
                         int64_t* offsets, int32_t* recv_from) {
  if (n_ranks < 1 || rank < 0 || rank >= n_ranks || root < 0 || root >= n_ranks || send_bytes < 0 || !recv_from)
    return -slg_internal_fail(SLG_ERR_INVALID, "bad gatherv argument");
  if (rank != root) {
    recv_from[0] = send_bytes > 0;
    return send_bytes > 0;                     // the root skips zero-byte peers too
  }
  if (!recv_bytes || !offsets) return -slg_internal_fail(SLG_ERR_INVALID, "root needs recv_bytes, offsets");
  if (recv_bytes[root] != send_bytes) return -slg_internal_fail(SLG_ERR_INVALID, "recv_bytes[root] != send_bytes");
  int32_t ops = 0;
  offsets[0] = 0;
  for (int32_t r = 0; r < n_ranks; ++r) {
    if (recv_bytes[r] < 0) return -slg_internal_fail(SLG_ERR_INVALID, "negative recv_bytes");
    offsets[r + 1] = offsets[r] + recv_bytes[r];
    recv_from[r] = (r != root && recv_bytes[r] > 0);
    ops += recv_from[r];
  }
  return ops;
}

int32_t slg_gatherv(slg_gather_comm* g, const void* send, int64_t send_bytes, void* recv, const int64_t* recv_bytes,
                    int32_t root, void* stream) {
  if (!g || (send_bytes > 0 && !send)) return slg_internal_fail(SLG_ERR_INVALID, "bad gatherv argument");
  std::vector<int64_t> off(size_t(g->n_ranks) + 1, 0);
  std::vector<int32_t> from(size_t(g->n_ranks), 0);
  const int32_t ops = slg_gatherv_plan(g->n_ranks, g->rank, root, send_bytes, recv_bytes, off.data(), from.data());
  if (ops < 0) return -ops;
  RcclApi* a = rccl();
  if (!a) return slg_internal_fail(SLG_ERR_UNSUPPORTED, "RCCL (librccl.so.1) not found");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (g->rank != root) {
    if (!ops) return SLG_OK;
    const ncclResult_t r = a->send(send, size_t(send_bytes), ncclUint8, root, g->comm, s);
    return r == ncclSuccess ? SLG_OK : nccl_fail(a, r, "ncclSend");
  }
  if (off[size_t(g->n_ranks)] > 0 && !recv) return slg_internal_fail(SLG_ERR_INVALID, "root needs recv");
  char* dst = static_cast<char*>(recv);
  if (send_bytes > 0 && hipMemcpyAsync(dst + off[size_t(root)], send, size_t(send_bytes), hipMemcpyDeviceToDevice, s) != hipSuccess)
    return slg_internal_fail(SLG_ERR_HIP, "hipMemcpyAsync (root's own part) failed");
  if (!ops) return SLG_OK;
  ncclResult_t r = a->group_start();
  if (r != ncclSuccess) return nccl_fail(a, r, "ncclGroupStart");
  for (int p = 0; p < g->n_ranks; ++p) {
    if (!from[size_t(p)]) continue;
    r = a->recv(dst + off[size_t(p)], size_t(recv_bytes[p]), ncclUint8, p, g->comm, s);
    if (r != ncclSuccess) { a->group_end(); return nccl_fail(a, r, "ncclRecv"); }
  }
  r = a->group_end();
  if (r != ncclSuccess) return nccl_fail(a, r, "ncclGroupEnd");
  return SLG_OK;
}

int32_t slg_gather_destroy(slg_gather_comm* g) {
  if (!g) return SLG_OK;
  RcclApi* a = rccl();
  const ncclResult_t r = a ? a->comm_destroy(g->comm) : ncclSuccess;
  delete g;
  if (a && r != ncclSuccess) return nccl_fail(a, r, "ncclCommDestroy");
  return SLG_OK;
}

}  // extern "C"
