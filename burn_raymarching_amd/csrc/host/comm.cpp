// librm_host.so, part 4: the data-parallel collectives of the multi-rank training driver
// (SURVEY.md §8(e)): an RCCL communicator over xGMI, one process per GPU.
//
// The driver needs exactly two collectives, both on fp32 device buffers on its stream:
//   * a sum all-reduce of the packed activated-space gradient + the loss sum (7M+5 floats)
//     between rm_train_step and rm_optimizer_step, every step (train.rs:182-198);
//   * a broadcast from rank 0 of the next generation after prune_and_split (its size, then the
//     packed parameters) between stages (training.rs:87-238, train.rs:300-328).
// Both are latency-bound messages (0.2-115 KB), so RCCL's default algorithms are used as is.
//
// Rendezvous: rank 0 creates the ncclUniqueId and publishes it in a file (written to a
// temporary name and renamed, so readers never see a partial id); the other ranks poll for it.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

#include "rmh_common.hpp"

using namespace rmh;

namespace {

struct Rccl {
  ncclComm_t comm = nullptr;
};

int nccl_fail(ncclResult_t r, const char* what) {
  return fail(RMH_ERR_GPU, "%s: %s", what, ncclGetErrorString(r));
}

int rccl_all_reduce(void* state, float* buf, int64_t count, void* stream) {
  auto* s = static_cast<Rccl*>(state);
  const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, ncclFloat32, ncclSum, s->comm, (hipStream_t)stream);
  return r == ncclSuccess ? RMH_OK : nccl_fail(r, "ncclAllReduce");
}

int rccl_broadcast(void* state, float* buf, int64_t count, int32_t root, void* stream) {
  auto* s = static_cast<Rccl*>(state);
  const ncclResult_t r = ncclBroadcast(buf, buf, (size_t)count, ncclFloat32, root, s->comm, (hipStream_t)stream);
  return r == ncclSuccess ? RMH_OK : nccl_fail(r, "ncclBroadcast");
}

void rccl_abort(void* state) {
  auto* s = static_cast<Rccl*>(state);
  if (s && s->comm) {
    (void)ncclCommAbort(s->comm);  // pending and later collectives of the other ranks fail
    s->comm = nullptr;
  }
}

// The id file, if it was written at or after `since` (seconds since the epoch): a file left by
// an earlier run is not this run's id.
bool read_id(const std::string& path, ncclUniqueId& id, double since) {
  struct stat st;
  if (stat(path.c_str(), &st) != 0) return false;
  const double mtime = (double)st.st_mtim.tv_sec + 1e-9 * (double)st.st_mtim.tv_nsec;
  if (mtime < since) return false;
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  const size_t n = std::fread(&id, 1, sizeof id, f);
  std::fclose(f);
  return n == sizeof id;
}

}  // namespace

extern "C" {

int rmh_collective_rccl_create(int32_t rank, int32_t world, int32_t device, const char* id_path, double timeout_s,
                               rmh_collective* out) {
  if (!out || world < 1 || rank < 0 || rank >= world || (world > 1 && !id_path))
    return fail(RMH_ERR_INVALID_ARG, "bad collective arguments (rank %d, world %d)", rank, world);
  std::memset(out, 0, sizeof *out);
  if (hipSetDevice(device) != hipSuccess) return fail(RMH_ERR_GPU, "hipSetDevice(%d) failed", device);
  ncclUniqueId id;
  ncclResult_t r;
  // this rank's start (1 s of slack for file-system timestamp granularity and clock skew)
  const double since = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count() - 1.0;
  if (rank == 0) {
    if (world > 1) unlink(id_path);  // an earlier run's id: never this run's
    if ((r = ncclGetUniqueId(&id)) != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
    if (world > 1) {
      const std::string tmp = std::string(id_path) + ".tmp";
      FILE* f = std::fopen(tmp.c_str(), "wb");
      if (!f || std::fwrite(&id, 1, sizeof id, f) != sizeof id || std::fclose(f) != 0)
        return fail(RMH_ERR_IO, "cannot write the RCCL id to %s", tmp.c_str());
      if (std::rename(tmp.c_str(), id_path) != 0) return fail(RMH_ERR_IO, "cannot rename %s", tmp.c_str());
    }
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    while (!read_id(id_path, id, since)) {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
        return fail(RMH_ERR_IO, "rank %d: no RCCL id at %s after %.0f s", rank, id_path, timeout_s);
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
  }
  auto* s = new Rccl;
  if ((r = ncclCommInitRank(&s->comm, world, id, rank)) != ncclSuccess) {
    delete s;
    return nccl_fail(r, "ncclCommInitRank");
  }
  // every rank has joined (ncclCommInitRank is collective): the id file has served its purpose
  if (rank == 0 && world > 1) unlink(id_path);
  out->state = s;
  out->rank = rank;
  out->world = world;
  out->all_reduce_sum = rccl_all_reduce;
  out->broadcast = rccl_broadcast;
  out->abort = rccl_abort;
  return RMH_OK;
}

void rmh_collective_rccl_destroy(rmh_collective* c) {
  if (!c || !c->state) return;
  auto* s = static_cast<Rccl*>(c->state);
  if (s->comm) (void)ncclCommDestroy(s->comm);
  delete s;
  c->state = nullptr;
}

}  // extern "C"
