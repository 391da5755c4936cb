"""Debug: per-step march t (GPU vs fp32/fp64 oracle) to locate non-finite values."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from oracle import oracle as orc
from burn_raymarching_amd import render, model
sc = model.synthetic_scene(8, 1)
eye, tgt, fov = model.ring_cameras(7)[1]
o, d = orc.camera_rays(64, 64, eye, tgt, fov, precision='f32')
s = model.scene_tensors(sc)
O, D = torch.from_numpy(o).cuda(), torch.from_numpy(d).cuda()
for S in [1, 2, 4, 8, 12, 16, 20, 24, 28, 32, 36, 40]:
    out, t = render.render_diff_forward(O, D, s, 5.0, S, return_t=True)
    out = out.cpu().numpy(); t = t.cpu().numpy()
    r32, t32 = orc.render_diff(o, d, sc, S, 5.0, precision='f32', with_t=True)
    r64, t64 = orc.render_diff(o.astype(np.float64), d.astype(np.float64), sc, S, 5.0, precision='f64', with_t=True)
    bad = ~np.isfinite(t)
    print(f"S={S:3d} t nonfinite={bad.sum():5d} out nonfinite={(~np.isfinite(out)).sum():5d} "
          f"max|t-t64|={np.nanmax(np.abs(t-t64)):.3e} max t64={t64.max():.3e} max|t32-t64|={np.abs(t32-t64).max():.3e} "
          f"out err={np.nanmax(np.abs(out-r64)):.3e} out32 err={np.abs(r32-r64).max():.3e}")
    if bad.any():
        i = np.argmax(bad); print('  first bad ray', i, 't64', t64[i], 't32', t32[i])
