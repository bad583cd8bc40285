// Gradient all-reduce over RCCL (xGMI), the data-parallel exchange of the training step
// (reference: Lightning `strategy: ddp`, mr_gen/model/lstmformer/config.yaml:127 — one process
// per GPU, gradients averaged across ranks after backward; SURVEY §8b `mrg_comm_*`, §8e).
//
// The C-ABI owns one RCCL communicator per handle.  RCCL is resolved at run time (dlopen of the
// `librccl.so.1` SONAME, RTLD_NOLOAD first), so the library torch already mapped is the one used
// (one RCCL per process, like the one HIP runtime: SURVEY §7) and libmrg.so still loads on a host
// with no RCCL at all.  The unique id is 128 opaque bytes (ncclUniqueId) that the host side moves
// between ranks over any channel (torch.distributed's store in ddp.NativeComm).
//
// Every call is stream-ordered on the hipStream_t the caller passes; nothing synchronises the
// device, so an all-reduce can sit on a communication stream beside the backward.
#include "mrg_common.h"
#include <dlfcn.h>
#include <mutex>

namespace {

// RCCL ABI subset (rccl.h, NCCL 2.x ABI): opaque comm pointer, 128-byte unique id, enums.
typedef struct { char internal[128]; } RcclUniqueId;
typedef void* RcclComm;
enum { kRcclFloat32 = 7 };               // ncclFloat32
enum { kRcclSum = 0, kRcclAvg = 4 };     // ncclSum, ncclAvg

struct Rccl {
  int (*get_unique_id)(RcclUniqueId*) = nullptr;
  int (*comm_init_rank)(RcclComm*, int, RcclUniqueId, int) = nullptr;
  int (*comm_destroy)(RcclComm) = nullptr;
  int (*all_reduce)(const void*, void*, size_t, int, int, RcclComm, hipStream_t) = nullptr;
  int (*group_start)() = nullptr;
  int (*group_end)() = nullptr;
  const char* (*error_string)(int) = nullptr;
  void* handle = nullptr;
  bool ok = false;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    r.handle = h;
    r.get_unique_id = (int (*)(RcclUniqueId*))dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (int (*)(RcclComm*, int, RcclUniqueId, int))dlsym(h, "ncclCommInitRank");
    r.comm_destroy = (int (*)(RcclComm))dlsym(h, "ncclCommDestroy");
    r.all_reduce = (int (*)(const void*, void*, size_t, int, int, RcclComm, hipStream_t))dlsym(h, "ncclAllReduce");
    r.group_start = (int (*)())dlsym(h, "ncclGroupStart");
    r.group_end = (int (*)())dlsym(h, "ncclGroupEnd");
    r.error_string = (const char* (*)(int))dlsym(h, "ncclGetErrorString");
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_reduce && r.group_start && r.group_end;
  });
  return r;
}

const char* rccl_err(int code) {
  Rccl& r = rccl();
  return r.error_string ? r.error_string(code) : "rccl error";
}

}  // namespace

#define MRG_RCCL(call)                                                                  \
  do {                                                                                  \
    int _c = (call);                                                                    \
    if (_c != 0) {                                                                      \
      ::mrg::set_error("%s failed: %s (%d)", #call, rccl_err(_c), _c);                  \
      return 5;                                                                         \
    }                                                                                   \
  } while (0)

// 1 if an RCCL library could be resolved in this process, else 0.
MRG_API int mrg_comm_available() { return rccl().ok ? 1 : 0; }

// Bytes of the opaque unique id (ncclUniqueId).
MRG_API size_t mrg_comm_id_bytes() { return sizeof(RcclUniqueId); }

// Rank 0 creates the id; the caller broadcasts the bytes to every rank.
MRG_API int mrg_comm_unique_id(void* id_out) {
  MRG_REQUIRE(id_out, "mrg_comm_unique_id: null output");
  Rccl& r = rccl();
  MRG_REQUIRE(r.ok, "mrg_comm_unique_id: librccl.so.1 not found in this process");
  RcclUniqueId id;
  MRG_RCCL(r.get_unique_id(&id));
  memcpy(id_out, &id, sizeof(id));
  return 0;
}

// Collective over all ranks (each on its own GPU, selected by the caller with hipSetDevice /
// torch.cuda.set_device before this call).  *comm_out receives the handle.
MRG_API int mrg_comm_init(void** comm_out, int nranks, const void* id, int rank) {
  MRG_REQUIRE(comm_out && id, "mrg_comm_init: null argument");
  MRG_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "mrg_comm_init: rank %d of %d", rank, nranks);
  Rccl& r = rccl();
  MRG_REQUIRE(r.ok, "mrg_comm_init: librccl.so.1 not found in this process");
  RcclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  RcclComm c = nullptr;
  MRG_RCCL(r.comm_init_rank(&c, nranks, uid, rank));
  *comm_out = c;
  return 0;
}

// In-place fp32 all-reduce of `nbuckets` spans of one buffer, issued as one RCCL group on
// `stream`: op 0 = sum, 1 = mean (ncclAvg).  Buckets let the caller send the flat gradient
// buffer in reverse-layer slices as the backward produces them.
MRG_API int mrg_comm_allreduce_f32(void* comm, float* buf, const long* offsets, const long* counts, int nbuckets,
                                   int op, hipStream_t stream) {
  MRG_REQUIRE(comm && buf && offsets && counts && nbuckets >= 1, "mrg_comm_allreduce_f32: bad arguments");
  MRG_REQUIRE(op == 0 || op == 1, "mrg_comm_allreduce_f32: op must be 0 (sum) or 1 (mean)");
  Rccl& r = rccl();
  MRG_REQUIRE(r.ok, "mrg_comm_allreduce_f32: librccl.so.1 not found in this process");
  MRG_RCCL(r.group_start());
  for (int i = 0; i < nbuckets; ++i) {
    if (counts[i] <= 0) continue;
    float* p = buf + offsets[i];
    int c = r.all_reduce(p, p, (size_t)counts[i], kRcclFloat32, op == 1 ? kRcclAvg : kRcclSum, (RcclComm)comm,
                         stream);
    if (c != 0) {
      r.group_end();
      mrg::set_error("ncclAllReduce failed: %s (%d)", rccl_err(c), c);
      return 5;
    }
  }
  MRG_RCCL(r.group_end());
  return 0;
}

MRG_API int mrg_comm_destroy(void* comm) {
  if (!comm) return 0;
  Rccl& r = rccl();
  MRG_REQUIRE(r.ok, "mrg_comm_destroy: librccl.so.1 not found in this process");
  MRG_RCCL(r.comm_destroy((RcclComm)comm));
  return 0;
}
