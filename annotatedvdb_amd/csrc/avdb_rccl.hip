// Node exchange in the C ABI (SURVEY.md §8b `avdb_hist_allgather`): every rank's
// L8 histogram and counters all-gathered over RCCL (xGMI between the GPUs of a
// node) and summed per bin on the device, so a caller that binds only
// libavdb_hip.so — not torch.distributed — can do the one collective of the
// path (§8e).  The reference has no collective at all: one OS process per
// chromosome file (Load/bin/load_vcf_file.py:307-313); this replaces its
// per-file log summaries with node totals.
//
// RCCL is opened with dlopen at first use: the library has no link-time RCCL
// dependency, and a process that already holds an RCCL (torch's) shares it.
#include "avdb_internal.hpp"

#include <dlfcn.h>
#include <mutex>
#include <rccl/rccl.h>
#include <string.h>

namespace {

struct Rccl {
  void* h = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclCommCount) comm_count = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl* rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names) {
      r.h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
      if (r.h) break;
    }
    if (!r.h) return;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(r.h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(r.h, "ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(r.h, "ncclCommDestroy"));
    r.comm_count = reinterpret_cast<decltype(r.comm_count)>(dlsym(r.h, "ncclCommCount"));
    r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(r.h, "ncclAllGather"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(r.h, "ncclGetErrorString"));
  });
  if (!r.h || !r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.comm_count || !r.all_gather)
    return nullptr;
  return &r;
}

#define AVDB_RCCL_TRY(R, expr)                                                           \
  do {                                                                                   \
    const ncclResult_t _r = (expr);                                                      \
    if (_r != ncclSuccess) {                                                             \
      avdb_set_error("%s failed: %s", #expr, (R)->error_string ? (R)->error_string(_r) : "?"); \
      return AVDB_ERCCL;                                                                 \
    }                                                                                    \
  } while (0)

// per-rank slot: the histogram (u32, padded to 8 bytes) then the counters (u64)
inline size_t slot_bytes(size_t n_bins, size_t n_counters) {
  return ((4 * n_bins + 7) & ~size_t(7)) + 8 * n_counters;
}

// node totals: bin b (and counter c) summed over the world's slots
__global__ __launch_bounds__(avdb::kBlock) void k_sum_ranks(const uint8_t* __restrict__ slots, int world,
                                                            size_t slot, size_t n_bins, size_t n_counters,
                                                            uint32_t* __restrict__ node_hist,
                                                            unsigned long long* __restrict__ node_counters) {
  const size_t hist_bytes = (4 * n_bins + 7) & ~size_t(7);
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n_bins + n_counters;
       i += size_t(gridDim.x) * blockDim.x) {
    if (i < n_bins) {
      uint32_t s = 0;
      for (int r = 0; r < world; ++r) s += reinterpret_cast<const uint32_t*>(slots + size_t(r) * slot)[i];
      node_hist[i] = s;
    } else {
      const size_t c = i - n_bins;
      unsigned long long s = 0;
      for (int r = 0; r < world; ++r)
        s += reinterpret_cast<const unsigned long long*>(slots + size_t(r) * slot + hist_bytes)[c];
      node_counters[c] = s;
    }
  }
}

}  // namespace

extern "C" int avdb_rccl_unique_id(void* id) {
  if (!id) { avdb_set_error("avdb_rccl_unique_id: null argument"); return AVDB_EINVAL; }
  const Rccl* R = rccl();
  if (!R) { avdb_set_error("avdb_rccl_unique_id: RCCL (librccl.so) could not be loaded"); return AVDB_ERCCL; }
  ncclUniqueId u;
  AVDB_RCCL_TRY(R, R->get_unique_id(&u));
  memcpy(id, &u, sizeof(u));
  return AVDB_OK;
}

extern "C" int avdb_rccl_comm_init(avdb_ctx* ctx, int world, int rank, const void* id, void** comm) {
  if (!ctx || !id || !comm || world < 1 || rank < 0 || rank >= world) {
    avdb_set_error("avdb_rccl_comm_init: bad argument");
    return AVDB_EINVAL;
  }
  const Rccl* R = rccl();
  if (!R) { avdb_set_error("avdb_rccl_comm_init: RCCL (librccl.so) could not be loaded"); return AVDB_ERCCL; }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  AVDB_RCCL_TRY(R, R->comm_init_rank(&c, world, u, rank));
  *comm = c;
  return AVDB_OK;
}

extern "C" int avdb_rccl_comm_destroy(void* comm) {
  if (!comm) return AVDB_OK;
  const Rccl* R = rccl();
  if (!R) { avdb_set_error("avdb_rccl_comm_destroy: RCCL (librccl.so) could not be loaded"); return AVDB_ERCCL; }
  AVDB_RCCL_TRY(R, R->comm_destroy(static_cast<ncclComm_t>(comm)));
  return AVDB_OK;
}

extern "C" int avdb_hist_allgather_workspace_size(int world, size_t n_bins, size_t n_counters, size_t* bytes) {
  if (!bytes || world < 1) { avdb_set_error("avdb_hist_allgather_workspace_size: bad argument"); return AVDB_EINVAL; }
  *bytes = size_t(world + 1) * slot_bytes(n_bins, n_counters);
  return AVDB_OK;
}

extern "C" int avdb_hist_allgather(avdb_ctx* ctx, void* comm, const uint32_t* hist, size_t n_bins,
                                   const uint64_t* counters, size_t n_counters, uint32_t* node_hist,
                                   uint64_t* node_counters, void* workspace, size_t workspace_bytes,
                                   void* stream) {
  if (!ctx || !comm || (n_bins && (!hist || !node_hist)) || (n_counters && (!counters || !node_counters))) {
    avdb_set_error("avdb_hist_allgather: null argument");
    return AVDB_EINVAL;
  }
  const Rccl* R = rccl();
  if (!R) { avdb_set_error("avdb_hist_allgather: RCCL (librccl.so) could not be loaded"); return AVDB_ERCCL; }
  int world = 0;
  AVDB_RCCL_TRY(R, R->comm_count(static_cast<ncclComm_t>(comm), &world));
  size_t need = 0;
  avdb_hist_allgather_workspace_size(world, n_bins, n_counters, &need);
  if (!workspace || workspace_bytes < need || reinterpret_cast<uintptr_t>(workspace) % 8) {
    avdb_set_error("avdb_hist_allgather: 8-byte aligned workspace of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  if (n_bins + n_counters == 0) return AVDB_OK;
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t slot = slot_bytes(n_bins, n_counters);
  const size_t hist_bytes = (4 * n_bins + 7) & ~size_t(7);
  uint8_t* send = static_cast<uint8_t*>(workspace);
  uint8_t* recv = send + slot;
  if (n_bins) AVDB_HIP_TRY(hipMemcpyAsync(send, hist, 4 * n_bins, hipMemcpyDeviceToDevice, s));
  if (n_counters) AVDB_HIP_TRY(hipMemcpyAsync(send + hist_bytes, counters, 8 * n_counters, hipMemcpyDeviceToDevice, s));
  // one collective: every rank's slot, in rank order
  AVDB_RCCL_TRY(R, R->all_gather(send, recv, slot, ncclUint8, static_cast<ncclComm_t>(comm), s));
  const unsigned grid = stream_grid(n_bins + n_counters, avdb::kBlock, 256);
  hipLaunchKernelGGL(k_sum_ranks, dim3(grid), dim3(avdb::kBlock), 0, s, recv, world, slot, n_bins, n_counters,
                     node_hist, reinterpret_cast<unsigned long long*>(node_counters));
  AVDB_LAUNCH_CHECK("k_sum_ranks");
  return AVDB_OK;
}
