"""Workload for PMC probes: forward render_diff (camera mode) at the metric view size, repeated.

    RM_NO_EARLY_EXIT=1 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-trace -d out -- python3 tools/pmc_probe.py [S] [mode]

mode "fwd" (default) or "train"; S = march steps (32).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from burn_raymarching_amd import model, render  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    mode = sys.argv[2] if len(sys.argv) > 2 else "fwd"
    sc = model.scene_tensors(model.synthetic_scene(256, 0))
    cams = model.ring_cameras(10)[:2]
    tgt = render.render_diff_camera(cams, 512, 512, model.scene_tensors(model.synthetic_scene(256, 1)), 32.0, S)
    for _ in range(5):
        if mode == "fwd":
            render.render_diff_camera(cams, 512, 512, sc, 32.0, S)
        else:
            render.train_step_camera(cams, 512, 512, tgt, sc, 32.0, 0.5, S)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
