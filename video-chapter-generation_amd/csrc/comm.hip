// Gradient-exchange C ABI over RCCL (vcg_comm_init / vcg_allreduce_bucket).
//
// Replaces the NCCL communicator that DDP(model) builds inside reference train_video_segment_ddp.py:64-86,148
// (one process per GPU, bucketed all-reduce of the gradients on every backward). One communicator per process
// (one process per GPU); every call is stream-ordered and asynchronous on the stream it is given, so a caller
// overlaps the exchange with the backward by issuing it on a side stream that waits for the bucket's producer.
//
// RCCL is resolved at run time with dlopen: the library already mapped into the process (PyTorch-ROCm ships and
// loads librccl.so.1 for its own "nccl" backend) is reused, so there is ONE RCCL per process; otherwise
// /opt/rocm/lib/librccl.so.1 is loaded. No CUDA/NCCL shim: rccl.h's types, RCCL's own entry points.
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <string.h>

#include <mutex>

#include "common.h"

namespace vcg {
namespace {

typedef ncclResult_t (*fn_get_uid)(ncclUniqueId*);
typedef ncclResult_t (*fn_init_rank)(ncclComm_t*, int, ncclUniqueId, int);
typedef ncclResult_t (*fn_all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                                      hipStream_t);
typedef ncclResult_t (*fn_broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
typedef ncclResult_t (*fn_destroy)(ncclComm_t);
typedef const char* (*fn_err)(ncclResult_t);

struct Rccl {
  void* handle = nullptr;
  fn_get_uid get_uid = nullptr;
  fn_init_rank init_rank = nullptr;
  fn_all_reduce all_reduce = nullptr;
  fn_broadcast broadcast = nullptr;
  fn_destroy destroy = nullptr;
  fn_err err = nullptr;
  const char* path = "";
};

Rccl g_rccl;
std::mutex g_mu;
ncclComm_t g_comm = nullptr;
int g_rank = -1, g_world = 0;

bool load_rccl() {
  if (g_rccl.handle) return true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // the process's RCCL (PyTorch's), if mapped
  g_rccl.path = "librccl.so.1 (already loaded)";
  if (!h) {
    h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    g_rccl.path = "/opt/rocm/lib/librccl.so.1";
  }
  if (!h) {
    set_error(std::string("vcg_comm: cannot load RCCL: ") + dlerror());
    return false;
  }
  g_rccl.get_uid = (fn_get_uid)dlsym(h, "ncclGetUniqueId");
  g_rccl.init_rank = (fn_init_rank)dlsym(h, "ncclCommInitRank");
  g_rccl.all_reduce = (fn_all_reduce)dlsym(h, "ncclAllReduce");
  g_rccl.broadcast = (fn_broadcast)dlsym(h, "ncclBroadcast");
  g_rccl.destroy = (fn_destroy)dlsym(h, "ncclCommDestroy");
  g_rccl.err = (fn_err)dlsym(h, "ncclGetErrorString");
  if (!g_rccl.get_uid || !g_rccl.init_rank || !g_rccl.all_reduce || !g_rccl.broadcast || !g_rccl.destroy ||
      !g_rccl.err) {
    set_error("vcg_comm: RCCL lacks an entry point (ncclGetUniqueId / CommInitRank / AllReduce / Broadcast)");
    return false;
  }
  g_rccl.handle = h;
  return true;
}

int rccl_status(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return VCG_OK;
  set_error(std::string(what) + ": " + (g_rccl.err ? g_rccl.err(r) : "RCCL error"));
  return VCG_ERR_HIP;
}

bool rccl_dtype(int dtype, ncclDataType_t* out) {
  if (dtype == VCG_F32) *out = ncclFloat32;
  else if (dtype == VCG_BF16) *out = ncclBfloat16;
  else return false;
  return true;
}

}  // namespace
}  // namespace vcg

// 128-byte communicator id (rank 0 creates it; the caller hands it to every rank, e.g. through its TCP store).
VCG_API int vcg_comm_unique_id(void* uid_out, int uid_bytes) {
  VCG_REQUIRE(uid_out != nullptr && uid_bytes >= (int)sizeof(ncclUniqueId), "uid buffer must hold 128 bytes");
  std::lock_guard<std::mutex> lk(vcg::g_mu);
  if (!vcg::load_rccl()) return VCG_ERR_UNSUPPORTED;
  ncclUniqueId id;
  const int rc = vcg::rccl_status(vcg::g_rccl.get_uid(&id), "ncclGetUniqueId");
  if (rc == VCG_OK) memcpy(uid_out, &id, sizeof(id));
  return rc;
}

// Collective: every rank calls it with the same uid; the current HIP device must be this rank's GPU.
VCG_API int vcg_comm_init(int rank, int world, const void* uid, int uid_bytes) {
  VCG_REQUIRE(world >= 1 && rank >= 0 && rank < world, "rank must be in [0, world)");
  VCG_REQUIRE(uid != nullptr && uid_bytes >= (int)sizeof(ncclUniqueId), "uid must hold 128 bytes");
  std::lock_guard<std::mutex> lk(vcg::g_mu);
  VCG_REQUIRE(vcg::g_comm == nullptr, "communicator already initialised (vcg_comm_finalize first)");
  if (!vcg::load_rccl()) return VCG_ERR_UNSUPPORTED;
  ncclUniqueId id;
  memcpy(&id, uid, sizeof(id));
  ncclComm_t c = nullptr;
  const int rc = vcg::rccl_status(vcg::g_rccl.init_rank(&c, world, id, rank), "ncclCommInitRank");
  if (rc != VCG_OK) return rc;
  vcg::g_comm = c;
  vcg::g_rank = rank;
  vcg::g_world = world;
  return VCG_OK;
}

VCG_API int vcg_comm_world(int* rank, int* world) {
  VCG_REQUIRE(vcg::g_comm != nullptr, "no communicator (vcg_comm_init)");
  if (rank) *rank = vcg::g_rank;
  if (world) *world = vcg::g_world;
  return VCG_OK;
}

// In-place SUM of `count` elements (VCG_F32 / VCG_BF16) at `ptr` across the ranks, enqueued on `s`.
VCG_API int vcg_allreduce_bucket(void* ptr, long long count, int dtype, hipStream_t s) {
  VCG_REQUIRE(vcg::g_comm != nullptr, "no communicator (vcg_comm_init)");
  VCG_REQUIRE(count >= 0, "negative count");
  if (count == 0) return VCG_OK;
  VCG_REQUIRE(ptr != nullptr, "null bucket");
  ncclDataType_t t;
  VCG_REQUIRE(vcg::rccl_dtype(dtype, &t), "dtype must be VCG_F32 or VCG_BF16");
  return vcg::rccl_status(vcg::g_rccl.all_reduce(ptr, ptr, (size_t)count, t, ncclSum, vcg::g_comm, s),
                          "ncclAllReduce");
}

// In-place broadcast from `root` (parameters / BatchNorm buffers, reference train_video_segment_ddp.py:261-263).
VCG_API int vcg_broadcast_bucket(void* ptr, long long count, int dtype, int root, hipStream_t s) {
  VCG_REQUIRE(vcg::g_comm != nullptr, "no communicator (vcg_comm_init)");
  VCG_REQUIRE(count >= 0 && root >= 0 && root < vcg::g_world, "bad count / root");
  if (count == 0) return VCG_OK;
  VCG_REQUIRE(ptr != nullptr, "null bucket");
  ncclDataType_t t;
  VCG_REQUIRE(vcg::rccl_dtype(dtype, &t), "dtype must be VCG_F32 or VCG_BF16");
  return vcg::rccl_status(vcg::g_rccl.broadcast(ptr, ptr, (size_t)count, t, root, vcg::g_comm, s), "ncclBroadcast");
}

VCG_API int vcg_comm_finalize(void) {
  std::lock_guard<std::mutex> lk(vcg::g_mu);
  if (vcg::g_comm == nullptr) return VCG_OK;
  const int rc = vcg::rccl_status(vcg::g_rccl.destroy(vcg::g_comm), "ncclCommDestroy");
  vcg::g_comm = nullptr;
  vcg::g_rank = -1;
  vcg::g_world = 0;
  return rc;
}
