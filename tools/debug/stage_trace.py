"""Debug: compare per-ray forward intermediates (rm_debug_intermediates) with the oracle."""
import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from oracle import oracle as orc
from burn_raymarching_amd import render, model, native
names = ['t', 'tf', 'nx', 'ny', 'nz', 'L', 'mr', 'mg', 'mb', 'Df', 'mu', 'ndotl', 'dmin', 'Zw', 'Zb', 'pad', 'D+x', 'D-x', 'D+y', 'D-y', 'D+z', 'D-z']
for (M, S, k, seed) in [(8, 1, 5.0, 1)]:
    sc = model.synthetic_scene(M, seed)
    eye, tgt, fov = model.ring_cameras(7)[seed]
    o, d = orc.camera_rays(64, 64, eye, tgt, fov, precision='f32')
    s = model.scene_tensors(sc)
    ctx = render.context()
    dbg = torch.zeros((o.shape[0], 24), device='cuda')
    O, D = torch.from_numpy(o).cuda(), torch.from_numpy(d).cuda()
    mp = native.march_params(S, k)
    ctx.check(ctx._lib.rm_debug_intermediates(ctx.handle, ctypes.c_void_p(O.data_ptr()), ctypes.c_void_p(D.data_ptr()), o.shape[0], ctypes.byref(s.c_struct()), ctypes.byref(mp), ctypes.c_void_p(dbg.data_ptr())), 'dbg')
    g = dbg.cpu().numpy().astype(np.float64)
    r64 = orc.render_diff_debug(o.astype(np.float64), d.astype(np.float64), sc, S, k, 'f64')
    r32 = orc.render_diff_debug(o, d, sc, S, k, 'f32').astype(np.float64)
    print(f'M={M} S={S} k={k}')
    for c, nm in enumerate(names):
        eg = np.abs(g[:, c] - r64[:, c]); e32 = np.abs(r32[:, c] - r64[:, c])
        i = np.argmax(eg)
        if nm == 'pad': continue
        print(f'  {nm:6s} gpu max {eg.max():.2e} mean {eg.mean():.2e} | f32 max {e32.max():.2e} | worst ray {i}: gpu {g[i,c]:.6g} f64 {r64[i,c]:.6g}')
