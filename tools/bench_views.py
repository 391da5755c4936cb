"""Train-kernel time per 512x512 view vs views per launch (occupancy / tail study)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from burn_raymarching_amd import model, render
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_parts import timed

W, M, S = 512, 256, 32
sc = model.scene_tensors(model.synthetic_scene(M, 0))
cams = model.ring_cameras(8)
tgt = render.render_diff_camera(cams, W, W, model.scene_tensors(model.synthetic_scene(M, 1)), 32.0, S)
ctx = render.context()
res = {}
for v in (1, 2, 4, 8):
    ms = timed(ctx, lambda: render.train_step_camera(cams[:v], W, W, tgt[:v * W * W], sc, 32.0, 0.5, S), reps=10)
    res[f"train_v{v}_ms_per_view"] = round(ms / v, 4)
    msf = timed(ctx, lambda: render.render_diff_camera(cams[:v], W, W, sc, 32.0, S), reps=10)
    res[f"fwd_v{v}_ms_per_view"] = round(msf / v, 4)
print(json.dumps(res))
