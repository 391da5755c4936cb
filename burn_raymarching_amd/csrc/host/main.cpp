// rm_train: command-line front end of librm_host.so, standing in for the reference's
// binaries (src/bin/train.rs, src/bin/generate.rs) on MI355X.
//
//   rm_train train    [--cameras data/cameras.json] [--out .] [--stages 5] [--steps 700]
//                     [--batch 16384] [--size 256x256] [--march-steps 40] [--seed 0]
//                     [--log-every 100] [--no-previews] [--device 0] [--ranks N]
//                     [--split-scale 1] [--split-move 0.05] [--split-all] [--max-spheres 0]
//                     [--color-f16]
//     --ranks N: data-parallel training on N GPUs (devices 0..N-1), one process per GPU over
//     RCCL: this process forks the N rank processes before anything touches a GPU and waits
//     for them. (--rank r --world N --comm-file F [--run-id S] [--comm-timeout SEC] run one rank
//     of a run launched elsewhere: every rank of the run gets the same F and S.)
//     --split-scale / --split-move: prune_and_split's split threshold scale and minimum move
//     (negative = no such condition; an explicit 0 is refused: rmh_train_config reads 0 as the
//     reference's 1 / 0.05, where rmh_prune_and_split_ex's 0 / 0 splits every sphere);
//     --split-all: every surviving sphere splits (both negative: growth runs such as BASELINE
//     configs[4]); --max-spheres caps the next generation, 0 = no cap;
//     --color-f16: fp16 colour / fp32 SDF.
//   rm_train generate [--out data] [--prefix data/] [--size 256x256] [--device 0]
//   rm_train preview  --scene scene.json --png out.png [--size 256x256]
//                     [--eye 0,0,-2.5] [--target 0,0,0] [--fov 50] [--radius-offset 0.01]
#include <signal.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rm_host.h"

namespace {

int usage() {
  std::fprintf(stderr,
               "usage: rm_train train|generate|preview [options]\n"
               "  train    --cameras F --out D --stages N --steps N --batch N --size WxH --march-steps N\n"
               "           --seed N --log-every N --no-previews --device N --ranks N\n"
               "           --split-scale F --split-move F --split-all --max-spheres N --color-f16\n"
               "           --rank R --world N --comm-file F --run-id S --comm-timeout SEC\n"
               "  generate --out D --prefix P --size WxH --device N\n"
               "  preview  --scene F --png F --size WxH --eye x,y,z --target x,y,z --fov F --radius-offset F\n");
  return 2;
}

bool parse_size(const char* s, int32_t& w, int32_t& h) { return std::sscanf(s, "%dx%d", &w, &h) == 2 && w > 0 && h > 0; }

bool parse_vec3(const char* s, float v[3]) { return std::sscanf(s, "%f,%f,%f", &v[0], &v[1], &v[2]) == 3; }

int report(int rc, const char* what) {
  if (rc != RMH_OK) std::fprintf(stderr, "rm_train %s: %s\n", what, rmh_last_error());
  return rc == RMH_OK ? 0 : 1;
}

// One rank of a data-parallel run: RCCL communicator, rmh_train, rank 0 prints the result.
int train_rank(rmh_train_config cfg, int rank, int world, const char* comm_file, const char* run_id,
               double comm_timeout) {
  rmh_collective comm;
  if (world > 1 || rank >= 0) {
    if (rmh_collective_rccl_create(rank, world, cfg.device, comm_file, run_id, comm_timeout, &comm) !=
        RMH_OK)
      return report(RMH_ERR_GPU, "train (RCCL)");
    cfg.comm = &comm;
  }
  rmh_train_result res;
  const int rc = rmh_train(&cfg, &res, nullptr, 0);
  if (cfg.comm) rmh_collective_rccl_destroy(&comm);
  if (rc == RMH_OK && rank <= 0)
  {
    // final_loss_bits: the loss's fp32 bit pattern, so that a run can be compared bit for bit
    uint32_t bits = 0;
    const float fl = (float)res.final_loss;
    std::memcpy(&bits, &fl, sizeof bits);
    std::printf("{\"num_spheres\": %d, \"steps\": %d, \"final_loss\": %.6g, \"final_loss_bits\": \"%08x\", "
                "\"seconds\": %.4f, \"step_ms\": %.4f, \"ranks\": %d}\n",
                res.num_spheres, res.steps, res.final_loss, bits, res.seconds, res.step_ms, world);
  }
  return report(rc, "train");
}

// --ranks N: one rank process per GPU (devices 0..N-1), forked before this process touches a
// GPU (no exec: each child runs its rank directly). Waits for all; when one fails the others
// are terminated. Returns the first failing exit status (0 if all succeed).
int launch_ranks(const rmh_train_config& cfg, int n, double comm_timeout) {
  char dir[] = "/tmp/rm_train_XXXXXX";
  if (!mkdtemp(dir)) {
    std::perror("mkdtemp");
    return 1;
  }
  const std::string id_file = std::string(dir) + "/rccl_id";
  char run_id[64];  // the directory is fresh already; the id makes the file's owner explicit
  std::snprintf(run_id, sizeof run_id, "rm_train-%d-%s", (int)getpid(), dir + 5);
  std::fflush(nullptr);
  std::vector<pid_t> pids;
  for (int r = 0; r < n; ++r) {
    const pid_t pid = fork();
    if (pid < 0) {
      std::perror("fork");
      for (pid_t p : pids) kill(p, SIGTERM);
      return 1;
    }
    if (pid == 0) {
      rmh_train_config c = cfg;
      c.device = r;
      const int code = train_rank(c, r, n, id_file.c_str(), run_id, comm_timeout);
      std::fflush(nullptr);
      _exit(code);
    }
    pids.push_back(pid);
  }
  int rc = 0;
  for (size_t left = pids.size(); left > 0; --left) {
    int status = 0;
    const pid_t p = wait(&status);
    if (p < 0) break;
    const int code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + (WIFSIGNALED(status) ? WTERMSIG(status) : 0);
    if (code != 0 && rc == 0) {
      rc = code;
      for (pid_t q : pids)
        if (q != p) kill(q, SIGTERM);
    }
  }
  unlink(id_file.c_str());
  unlink((id_file + ".tmp").c_str());
  rmdir(dir);
  return rc;
}

}  // namespace

#ifndef RMT_SOURCE_SHA
#define RMT_SOURCE_SHA "unknown"  // _build.py passes the sha256 of main.cpp and rm_host.h
#endif

int main(int argc, char** argv) {
  if (argc < 2) return usage();
  const std::string cmd = argv[1];
  if (cmd == "--version") {  // this program's sources, then the host library's (see rmh_version)
    std::printf("rm_train src " RMT_SOURCE_SHA "\n%s\n", rmh_version());
    return 0;
  }
  auto need = [&](int i) { return i + 1 < argc; };
  if (cmd == "train") {
    rmh_train_config cfg;
    rmh_train_config_default(&cfg);
    int ranks = 0, rank = -1, world = 1;
    bool device_given = false;
    const char* comm_file = nullptr;
    const char* run_id = nullptr;
    double comm_timeout = 300.0;
    for (int i = 2; i < argc; ++i) {
      const std::string a = argv[i];
      if (a == "--no-previews") {
        cfg.previews = 0;
      } else if (a == "--split-all") {  // every surviving sphere splits (configs[4] growth runs)
        cfg.split_scale = -1.0f;
        cfg.split_move = -1.0f;
      } else if (a == "--color-f16") {
        cfg.color_f16 = 1;
      } else if (!need(i)) {
        return usage();
      } else if (a == "--cameras") {
        cfg.cameras_json = argv[++i];
      } else if (a == "--out") {
        cfg.out_dir = argv[++i];
      } else if (a == "--stages") {
        cfg.stages = std::atoi(argv[++i]);
      } else if (a == "--steps") {
        cfg.steps_per_stage = std::atoi(argv[++i]);
      } else if (a == "--batch") {
        cfg.batch = std::atoi(argv[++i]);
      } else if (a == "--size") {
        if (!parse_size(argv[++i], cfg.width, cfg.height)) return usage();
      } else if (a == "--march-steps") {
        cfg.march_steps = std::atoi(argv[++i]);
      } else if (a == "--seed") {
        cfg.seed = std::strtoull(argv[++i], nullptr, 10);
      } else if (a == "--log-every") {
        cfg.log_every = std::atoi(argv[++i]);
      } else if (a == "--device") {
        cfg.device = std::atoi(argv[++i]);
        device_given = true;
      } else if (a == "--ranks") {
        ranks = std::atoi(argv[++i]);
      } else if (a == "--rank") {
        rank = std::atoi(argv[++i]);
      } else if (a == "--world") {
        world = std::atoi(argv[++i]);
      } else if (a == "--comm-file") {
        comm_file = argv[++i];
      } else if (a == "--run-id") {
        run_id = argv[++i];
      } else if (a == "--comm-timeout") {
        comm_timeout = std::atof(argv[++i]);
      } else if (a == "--split-scale" || a == "--split-move") {
        // 0 in rmh_train_config means "the reference value" (1 / 0.05), where prune_and_split_ex's
        // 0 / 0 splits every sphere: an explicit 0 here is refused so that an old "split everything"
        // command line cannot silently run the reference rule (use --split-all)
        const float v = (float)std::atof(argv[++i]);
        if (v == 0.0f) {
          std::fprintf(stderr, "%s 0 is ambiguous: use --split-all to split every sphere, or omit it for the "
                       "reference value\n", a.c_str());
          return 2;
        }
        (a == "--split-scale" ? cfg.split_scale : cfg.split_move) = v;
      } else if (a == "--max-spheres") {
        cfg.max_spheres = std::atoi(argv[++i]);
      } else {
        return usage();
      }
    }
    if (ranks > 0) return launch_ranks(cfg, ranks, comm_timeout);
    // one rank of a run launched elsewhere: without --device it takes LOCAL_RANK's device (or
    // its rank's): RCCL refuses two ranks on one device
    if (world > 1 && !device_given) {
      const char* lr = std::getenv("LOCAL_RANK");
      cfg.device = lr ? std::atoi(lr) : rank;
    }
    return train_rank(cfg, rank, world, comm_file, run_id, comm_timeout);
  }
  if (cmd == "generate") {
    const char* out = "data";
    const char* prefix = "data/";
    int32_t w = 256, h = 256, dev = 0;
    for (int i = 2; i < argc; ++i) {
      const std::string a = argv[i];
      if (!need(i)) return usage();
      if (a == "--out") out = argv[++i];
      else if (a == "--prefix") prefix = argv[++i];
      else if (a == "--size") {
        if (!parse_size(argv[++i], w, h)) return usage();
      } else if (a == "--device") dev = std::atoi(argv[++i]);
      else return usage();
    }
    return report(rmh_generate(out, prefix, w, h, dev), "generate");
  }
  if (cmd == "preview") {
    const char* scene = nullptr;
    const char* png = nullptr;
    int32_t w = 256, h = 256, dev = 0;
    float eye[3] = {0.0f, 0.0f, -2.5f}, tgt[3] = {0.0f, 0.0f, 0.0f}, fov = 50.0f, roff = 0.01f;
    for (int i = 2; i < argc; ++i) {
      const std::string a = argv[i];
      if (!need(i)) return usage();
      if (a == "--scene") scene = argv[++i];
      else if (a == "--png") png = argv[++i];
      else if (a == "--size") {
        if (!parse_size(argv[++i], w, h)) return usage();
      } else if (a == "--eye") {
        if (!parse_vec3(argv[++i], eye)) return usage();
      } else if (a == "--target") {
        if (!parse_vec3(argv[++i], tgt)) return usage();
      } else if (a == "--fov") fov = (float)std::atof(argv[++i]);
      else if (a == "--radius-offset") roff = (float)std::atof(argv[++i]);
      else if (a == "--device") dev = std::atoi(argv[++i]);
      else return usage();
    }
    if (!scene || !png) return usage();
    return report(rmh_preview(scene, png, w, h, eye, tgt, fov, roff, dev), "preview");
  }
  return usage();
}
