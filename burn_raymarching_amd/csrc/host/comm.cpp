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
// Rendezvous (rmh_rendezvous_*): rank 0 creates the ncclUniqueId and publishes it in a file
// (written to a temporary name and renamed, so readers never see a partial id) tagged with the
// run's id; the other ranks poll for a complete file with the same run id. No clock is involved:
// a rank may start, or finish its HIP initialisation, any time before the timeout. The id must
// name the run (not empty, not torchrun's default "none"), or a stale file could pass for it.
//
// Watchdog (rmh_collective.wait): a peer that died mid-run leaves the others spinning inside an
// RCCL kernel on their stream (over xGMI nothing reports the loss). The driver waits on its stream
// only through `wait`, which polls the stream and the communicator's asynchronous error, and
// aborts the communicator (ncclCommAbort ends its in-flight kernels) when the stream has not
// drained within the collective's timeout.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

#include "rmh_common.hpp"

using namespace rmh;

namespace {

constexpr char kMagic[8] = {'R', 'M', 'H', 'I', 'D', '0', '0', '2'};

struct Rccl {
  ncclComm_t comm = nullptr;
  double timeout_s = 300.0;
};

int nccl_fail(ncclResult_t r, const char* what) {
  return fail(RMH_ERR_GPU, "%s: %s", what, ncclGetErrorString(r));
}

int rccl_all_reduce(void* state, float* buf, int64_t count, void* stream) {
  auto* s = static_cast<Rccl*>(state);
  if (!s->comm) return fail(RMH_ERR_GPU, "ncclAllReduce: the communicator was aborted");
  const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, ncclFloat32, ncclSum, s->comm, (hipStream_t)stream);
  return r == ncclSuccess ? RMH_OK : nccl_fail(r, "ncclAllReduce");
}

int rccl_broadcast(void* state, float* buf, int64_t count, int32_t root, void* stream) {
  auto* s = static_cast<Rccl*>(state);
  if (!s->comm) return fail(RMH_ERR_GPU, "ncclBroadcast: the communicator was aborted");
  const ncclResult_t r = ncclBroadcast(buf, buf, (size_t)count, ncclFloat32, root, s->comm, (hipStream_t)stream);
  return r == ncclSuccess ? RMH_OK : nccl_fail(r, "ncclBroadcast");
}

// Frees this rank's communicator and ends its in-flight collectives. RCCL does not tell the
// peers: a peer blocked in a collective with this rank leaves it through its own watchdog
// (rccl_wait's timeout) or is ended by the launcher (rm_train --ranks terminates the others).
void rccl_abort(void* state) {
  auto* s = static_cast<Rccl*>(state);
  if (s && s->comm) {
    (void)ncclCommAbort(s->comm);
    s->comm = nullptr;
  }
}

int rccl_wait(void* state, void* stream) {
  auto* s = static_cast<Rccl*>(state);
  const auto t0 = std::chrono::steady_clock::now();
  for (int64_t polls = 0;; ++polls) {
    const hipError_t e = hipStreamQuery((hipStream_t)stream);
    if (e == hipSuccess) return RMH_OK;
    if (e != hipErrorNotReady) return fail(RMH_ERR_GPU, "hipStreamQuery: %s", hipGetErrorString(e));
    if (s && s->comm) {
      ncclResult_t async = ncclSuccess;
      if (ncclCommGetAsyncError(s->comm, &async) == ncclSuccess && async != ncclSuccess && async != ncclInProgress) {
        rccl_abort(s);
        return nccl_fail(async, "RCCL asynchronous error");
      }
    }
    const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (s && waited > s->timeout_s) {
      rccl_abort(s);  // ends this rank's pending collectives so the stream drains
      // the abort ends RCCL's kernels, not others': give the stream a bounded grace to drain and
      // return the error either way (an unbounded hipStreamSynchronize would hang the watchdog
      // itself behind a stuck non-collective kernel)
      const double grace = s->timeout_s < 10.0 ? s->timeout_s : 10.0;
      const auto ta = std::chrono::steady_clock::now();
      bool drained = false;
      while (!(drained = hipStreamQuery((hipStream_t)stream) != hipErrorNotReady) &&
             std::chrono::duration<double>(std::chrono::steady_clock::now() - ta).count() < grace)
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      return fail(RMH_ERR_GPU, "the stream did not drain within %.1f s (a peer rank left a collective?); "
                  "communicator aborted, stream %s", s->timeout_s,
                  drained ? "drained after the abort" : "still busy after the abort's grace period");
    }
    // spin briefly (the common case: a few microseconds of work left), then back off
    if (polls < 200) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(polls < 2000 ? 50 : 1000));
  }
}

std::string resolve_run_id(const char* run_id) {
  if (run_id) return run_id;
  for (const char* var : {"RMH_RUN_ID", "TORCHELASTIC_RUN_ID"}) {
    const char* v = std::getenv(var);
    if (v && *v) return v;
  }
  return std::string();
}

// A run id that names this run: not empty, and not torchrun's default "none" (every run launched
// without --rdzv-id has it). With such an id a file a crashed earlier run left at the same path
// would pass for this run's, and a rank that polls before rank 0 replaces it would join a dead
// ncclUniqueId (ncclCommInitRank has no timeout): the rendezvous refuses it.
int check_run_id(const std::string& id) {
  if (id.empty() || id == "none")
    return fail(RMH_ERR_INVALID_ARG,
                "the id-file rendezvous needs a run id naming this run (run_id, env RMH_RUN_ID or "
                "TORCHELASTIC_RUN_ID; got '%s'): a stale file of an earlier run could pass for this run's",
                id.c_str());
  return RMH_OK;
}

}  // namespace

extern "C" {

int rmh_rendezvous_publish(const char* path, const char* run_id, const void* blob, int64_t size) {
  if (!path || !blob || size < 0 || size > (1 << 20)) return fail(RMH_ERR_INVALID_ARG, "bad rendezvous arguments");
  const std::string id = resolve_run_id(run_id);
  if (const int rc = check_run_id(id)) return rc;
  std::string data(kMagic, sizeof kMagic);
  const uint32_t n = (uint32_t)id.size();
  const uint64_t sz = (uint64_t)size;
  data.append((const char*)&n, sizeof n).append(id).append((const char*)&sz, sizeof sz);
  data.append((const char*)blob, (size_t)size);
  unlink(path);  // an earlier run's file: never this run's
  const std::string tmp = std::string(path) + ".tmp";
  if (!write_file(tmp, data)) return fail(RMH_ERR_IO, "cannot write %s", tmp.c_str());
  if (std::rename(tmp.c_str(), path) != 0) return fail(RMH_ERR_IO, "cannot rename %s", tmp.c_str());
  return RMH_OK;
}

int rmh_rendezvous_read(const char* path, const char* run_id, void* blob, int64_t size, double timeout_s) {
  if (!path || !blob || size < 0) return fail(RMH_ERR_INVALID_ARG, "bad rendezvous arguments");
  const std::string id = resolve_run_id(run_id);
  if (const int rc = check_run_id(id)) return rc;
  const auto t0 = std::chrono::steady_clock::now();
  std::string seen;  // why the last file present was not taken (for the timeout message)
  for (;;) {
    std::string data;
    if (read_file(path, data)) {
      const size_t head = sizeof kMagic + sizeof(uint32_t);
      uint32_t n = 0;
      uint64_t sz = 0;
      if (data.size() < head || std::memcmp(data.data(), kMagic, sizeof kMagic) != 0) {
        seen = "not a rendezvous file";
      } else {
        std::memcpy(&n, data.data() + sizeof kMagic, sizeof n);
        if (data.size() < head + n + sizeof sz) {
          seen = "truncated";
        } else if (data.compare(head, n, id) != 0) {
          seen = "run id '" + data.substr(head, n) + "', expected '" + id + "'";
        } else {
          std::memcpy(&sz, data.data() + head + n, sizeof sz);
          if (sz != (uint64_t)size || data.size() != head + n + sizeof sz + sz) {
            seen = "wrong payload size";
          } else {
            std::memcpy(blob, data.data() + head + n + sizeof sz, (size_t)size);
            return RMH_OK;
          }
        }
      }
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      return fail(RMH_ERR_IO, "no rendezvous file for run '%s' at %s after %.1f s%s%s", id.c_str(), path, timeout_s,
                  seen.empty() ? "" : "; the file there: ", seen.c_str());
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

int rmh_collective_rccl_create(int32_t rank, int32_t world, int32_t device, const char* id_path, const char* run_id,
                               double timeout_s, rmh_collective* out) {
  if (!out || world < 1 || rank < 0 || rank >= world || (world > 1 && !id_path) || !(timeout_s > 0.0))
    return fail(RMH_ERR_INVALID_ARG, "bad collective arguments (rank %d, world %d)", rank, world);
  std::memset(out, 0, sizeof *out);
  if (world > 1) {  // before any GPU call: a launch without a run id fails at once
    if (const int rc = check_run_id(resolve_run_id(run_id))) {
      const std::string why = rmh_last_error();
      return fail(rc, "rank %d: %s", rank, why.c_str());
    }
  }
  if (hipSetDevice(device) != hipSuccess) return fail(RMH_ERR_GPU, "hipSetDevice(%d) failed", device);
  ncclUniqueId id;
  ncclResult_t r;
  int rc;
  if (rank == 0) {
    if ((r = ncclGetUniqueId(&id)) != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
    if (world > 1 && (rc = rmh_rendezvous_publish(id_path, run_id, &id, sizeof id)) != RMH_OK) return rc;
  } else if ((rc = rmh_rendezvous_read(id_path, run_id, &id, sizeof id, timeout_s)) != RMH_OK) {
    const std::string why = rmh_last_error();
    return fail(rc, "rank %d: %s", rank, why.c_str());
  }
  auto* s = new Rccl;
  s->timeout_s = timeout_s;
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
  out->wait = rccl_wait;
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
