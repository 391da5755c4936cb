"""Ray-mode debugging: the split train step of tests/test_gpu_split.py::test_split_continuation
with the continuation (default) and without (RM_SPLIT_CONT_STEPS=0): which rays' outputs differ."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from burn_raymarching_amd import model, native, render  # noqa: E402

W = H = 64
M, S, K = 300, 64, 32.0
sc = model.synthetic_scene(M, 23, radius_range=(0.02, 0.08))
s = model.scene_tensors(sc)
cams = model.ring_cameras(10, offset=3)[:2]
tg = render.render_diff_camera(cams, W, H, model.scene_tensors(model.synthetic_scene(M, 24)), K, S)
os.environ["RM_SPLIT"] = "1"


def run(env):
    for k in ("RM_SPLIT_CONT_STEPS",):
        os.environ.pop(k, None)
    os.environ.update(env)
    out = torch.empty_like(tg)
    loss, g, _ = render.train_step_camera(cams, W, H, tg, s, K, 0.3, S, out=out, march=native.march_params(S, K))
    torch.cuda.synchronize()
    return out.cpu().numpy(), {k: v.cpu().numpy() for k, v in g.items()}


a, ga = run({})
b, gb = run({"RM_SPLIT_CONT_STEPS": "0"})
c, gc = run({})
print("cont vs cont (determinism):", np.array_equal(a, c))
diff = np.nonzero(np.any(a != b, axis=1))[0]
print("rays differing:", len(diff), "of", len(a))
for i in diff[:20]:
    print(i, "group", i // 32, "lane", i % 32, a[i], b[i], tg.cpu().numpy()[i])
for k in ga:
    print(k, np.abs(ga[k] - gb[k]).max())
