// jr_comm.cpp — data-parallel gradient exchange over RCCL (xGMI), the
// collective half of libjr's C-ABI (jr_comm_init /
// jr_allreduce_sum / jr_comm_destroy).
//
// The reference has no collective call sites: its only multi-GPU path is an
// external tf_cnn_benchmarks parameter server (benchmarks.yaml.jinja.example:
// 81-90).  This replaces it with one RCCL communicator
// per process (one process per GPU): ncclAllReduce(sum) in place on the
// flat gradient (fp32 87.1 MB, or its bf16 copy 43.5 MB), enqueued on the
// caller's stream, so it can run on a dedicated comm stream beside the
// backward kernels and be captured in a HIP graph.  The unique id is either
// passed in (exchanged by the caller's own bootstrap) or handed over through
// a file (rank 0 writes it with an atomic rename, the others poll for it).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

#include "jr_common.h"

struct jr_comm {
  ncclComm_t comm;
  int rank, world;
};

namespace jr {

static int nccl_fail(ncclResult_t r, const char* what) {
  return fail(JR_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}

}  // namespace jr

using namespace jr;

static_assert(NCCL_UNIQUE_ID_BYTES == JR_COMM_ID_BYTES, "jr.h JR_COMM_ID_BYTES must match RCCL's id size");

JR_API int jr_comm_unique_id(uint8_t* id) {
  if (!id) return fail(JR_ERR_INVALID, "comm_unique_id: null output");
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
  std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return JR_OK;
}

JR_API int jr_comm_init(int rank, int world, const uint8_t* id, int device, jr_comm** out) {
  if (!out || !id || world <= 0 || rank < 0 || rank >= world || device < 0)
    return fail(JR_ERR_INVALID, "comm_init: bad arguments");
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return fail(JR_ERR_HIP, "comm_init: hipSetDevice failed");
  ncclUniqueId u;
  std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c;
  const ncclResult_t r = ncclCommInitRank(&c, world, u, rank);
  if (r != ncclSuccess) return nccl_fail(r, "ncclCommInitRank");
  *out = new jr_comm{c, rank, world};
  return JR_OK;
}

JR_API int jr_comm_init_file(int rank, int world, const char* uid_path, int device, int timeout_ms, jr_comm** out) {
  if (!uid_path || !out) return fail(JR_ERR_INVALID, "comm_init_file: bad arguments");
  uint8_t id[NCCL_UNIQUE_ID_BYTES];
  const std::string path(uid_path);
  if (rank == 0) {
    int rc = jr_comm_unique_id(id);
    if (rc) return rc;
    const std::string tmp = path + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return fail(JR_ERR_INVALID, "comm_init_file: cannot write " + tmp);
    const size_t w = std::fwrite(id, 1, sizeof(id), f);
    std::fclose(f);
    if (w != sizeof(id) || std::rename(tmp.c_str(), path.c_str()) != 0)
      return fail(JR_ERR_INVALID, "comm_init_file: cannot publish " + path);
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      FILE* f = std::fopen(path.c_str(), "rb");
      if (f) {
        const size_t n = std::fread(id, 1, sizeof(id), f);
        std::fclose(f);
        if (n == sizeof(id)) break;
      }
      const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0);
      if (timeout_ms >= 0 && ms.count() > timeout_ms) return fail(JR_ERR_INVALID, "comm_init_file: timed out waiting for " + path);
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
  }
  return jr_comm_init(rank, world, id, device, out);
}

JR_API int jr_allreduce_sum(jr_comm* comm, void* buf, size_t n, int dtype, void* stream) {
  if (!comm || (!buf && n)) return fail(JR_ERR_INVALID, "allreduce_sum: bad arguments");
  if (dtype != JR_F32 && dtype != JR_BF16) return fail(JR_ERR_INVALID, "allreduce_sum: dtype must be JR_F32 or JR_BF16");
  if (n == 0) return JR_OK;
  const ncclResult_t r = ncclAllReduce(buf, buf, n, dtype == JR_F32 ? ncclFloat32 : ncclBfloat16, ncclSum, comm->comm,
                                       as_stream(stream));
  if (r != ncclSuccess) return nccl_fail(r, "ncclAllReduce");
  return JR_OK;
}

JR_API int jr_comm_rank(const jr_comm* comm) { return comm ? comm->rank : -1; }
JR_API int jr_comm_world(const jr_comm* comm) { return comm ? comm->world : -1; }

JR_API int jr_comm_destroy(jr_comm* comm) {
  if (!comm) return JR_OK;
  const ncclResult_t r = ncclCommDestroy(comm->comm);
  delete comm;
  if (r != ncclSuccess) return nccl_fail(r, "ncclCommDestroy");
  return JR_OK;
}
