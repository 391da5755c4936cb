"""Run the reference's training schedule (rm_train train: train.rs:138-208 on the ten
data/cameras.json poses and target PNGs, seed 0) and print / write what pins its trajectory:
the final sphere count, the final loss's fp32 bits and the sha256 of the exported scene.json
(serde's shortest-round-trip floats: every parameter bit). One process and --ranks 1 (the
data-parallel step: sampled launch, RCCL all-reduce, update-only optimizer) must agree.

  python tools/pin_trajectory.py [--write tests/golden/rm_train_trajectory.json] [--log-every N]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "burn_raymarching_amd", "lib", "rm_train")
CAMS = os.path.join(ROOT, "tests", "golden", "cameras.json")


# BASELINE configs[4] as stated: the growth run of tools/gpu_configs.sh (the generate.rs targets at
# 512x512 on the cameras.json poses, 11 x 100 steps, every surviving sphere splits up to 4096,
# 128 march steps, fp16 colours) -- through the small kernel, the general kernel and the split march
# with its continuations, the fp16 optimizer and prune_and_split's growth knobs
GROWTH = ("--size", "512x512", "--march-steps", "128", "--color-f16", "--stages", "11", "--steps", "100",
          "--split-all", "--max-spheres", "4096")


def generate(out: str, timeout: float = 120.0) -> str:
    """rm_train generate at 512x512 into out/ (targets + cameras.json); returns the cameras path."""
    p = subprocess.run([EXE, "generate", "--out", out, "--prefix", "", "--size", "512x512"], capture_output=True,
                       text=True, timeout=timeout)
    if p.returncode != 0:
        raise RuntimeError(f"rm_train generate exited {p.returncode}: {p.stderr[-2000:]}")
    return os.path.join(out, "cameras.json")


def run(ranks: int = 0, log_every: int = 700, timeout: float = 300.0, extra=(), cams: str = CAMS):
    """One rm_train run; returns {num_spheres, final_loss_bits, scene_sha256, step_ms}."""
    with tempfile.TemporaryDirectory() as out:
        cmd = [EXE, "train", "--cameras", cams, "--out", out, "--no-previews", "--log-every", str(log_every)]
        if ranks:
            cmd += ["--ranks", str(ranks)]
        cmd += list(extra)
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
        if p.returncode != 0:
            raise RuntimeError(f"{' '.join(cmd)} exited {p.returncode}: {p.stderr[-2000:]}")
        res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
        with open(os.path.join(out, "scene.json"), "rb") as f:
            sha = hashlib.sha256(f.read()).hexdigest()
    return {"num_spheres": res["num_spheres"], "final_loss_bits": res["final_loss_bits"], "scene_sha256": sha,
            "final_loss": res["final_loss"], "step_ms": res["step_ms"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--write", default=None)
    ap.add_argument("--log-every", type=int, default=700)
    args = ap.parse_args()
    one = run(0, args.log_every)
    print("one process:", json.dumps(one), flush=True)
    r1 = run(1, args.log_every)
    print("--ranks 1:  ", json.dumps(r1), flush=True)
    keys = ("num_spheres", "final_loss_bits", "scene_sha256")
    if any(one[k] != r1[k] for k in keys):
        print("one process and --ranks 1 differ", file=sys.stderr)
        sys.exit(1)
    with tempfile.TemporaryDirectory() as data:
        cams = generate(data)
        g = run(0, 100, extra=GROWTH, cams=cams)
        print("growth:     ", json.dumps(g), flush=True)
        # the same run again, reading the loss only at the end: run-to-run determinism and the
        # loss readback's independence of the trajectory
        g2 = run(0, 1100, extra=GROWTH, cams=cams)
        print("growth (2): ", json.dumps(g2), flush=True)
    if any(g[k] != g2[k] for k in keys):
        print("the growth run is not reproducible", file=sys.stderr)
        sys.exit(1)
    if args.write:
        pin = {k: one[k] for k in keys}
        pin["final_loss"] = one["final_loss"]
        pin["what"] = ("rm_train train --cameras tests/golden/cameras.json --no-previews (seed 0): "
                       "train.rs:138-208's schedule, 5 x 700 steps, batch 16384; pinned by tools/pin_trajectory.py")
        pin["growth"] = {k: g[k] for k in keys + ("final_loss",)}
        pin["growth"]["what"] = "configs[4] growth run: rm_train generate --size 512x512, then train " + " ".join(GROWTH)
        with open(args.write, "w") as f:
            json.dump(pin, f, indent=1)
            f.write("\n")
        print("wrote", args.write)


if __name__ == "__main__":
    main()
