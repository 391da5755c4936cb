"""Driver: p_final points from the fp64 oracle -> GPU normal variants vs fp64 / fp32-CPU normals."""
import os, sys, struct, subprocess
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as orc
from burn_raymarching_amd.model import synthetic_scene, ring_cameras

def normal64(p, C, R, k, eps=np.float64(np.float32(1e-4)), dt=np.float64):
    p = p.astype(dt); C = C.astype(dt); R = R.astype(dt); k = dt(k); eps = dt(eps)
    D = []
    for a in range(3):
        for sg in (eps, -eps):
            tap = p.copy(); tap[:, a] = tap[:, a] + sg
            pp = (tap * tap).sum(1, keepdims=True); cc = (C * C).sum(1)[None]
            q = (pp + cc) - (tap @ C.T) * dt(2)
            d = np.sqrt(np.maximum(q, dt(1e-6))) - R[None]
            v = d * (-k); m = v.max(1, keepdims=True)
            s = np.exp(v - m).sum(1, keepdims=True)
            D.append(((np.log(np.maximum(s, dt(1e-8))) + m) / (-k))[:, 0])
    n = np.stack([D[0]-D[1], D[2]-D[3], D[4]-D[5]], 1)
    return n / np.sqrt((n*n).sum(1, keepdims=True) + dt(1e-6))

for (M, k, seed) in [(8, 5.0, 1), (64, 32.0, 2)]:
    sc = synthetic_scene(M, seed)
    eye, tgt, fov = ring_cameras(7)[seed]
    o, d = orc.camera_rays(64, 64, eye, tgt, fov, precision='f64')
    _, t = orc.render_diff(o, d, sc, 16, k, precision='f64', with_t=True)
    p = (o + d * t[:, None]).astype(np.float32)
    hit = np.linalg.norm(p, axis=1) < 1.0
    p = p[hit]
    n = len(p)
    path = os.path.join(HERE, 'pts.bin')
    with open(path, 'wb') as f:
        f.write(struct.pack('iif', n, M, k)); f.write(p.tobytes()); f.write(sc['centers'].astype(np.float32).tobytes()); f.write(sc['radius'].astype(np.float32).tobytes())
    subprocess.run([os.path.join(HERE, 'normal_variants'), path, path + '.out'], check=True)
    out = np.fromfile(path + '.out', np.float32).reshape(4, n, 3)
    ref = normal64(p, sc['centers'], sc['radius'], k)
    cpu32 = normal64(p, sc['centers'], sc['radius'], k, dt=np.float32)
    print(f'M={M} k={k} n={n}: cpu-f32 expansion err max {np.abs(cpu32-ref).max():.2e} mean {np.abs(cpu32-ref).mean():.2e}')
    for v, name in enumerate(['direct+v_sqrt+exp2/log2', 'direct+sqrt_rn+exp2/log2', 'expansion+v_sqrt+exp2/log2', 'direct+sqrt_rn+expf/logf']):
        e = np.abs(out[v] - ref)
        print(f'   {name:30s} max {e.max():.2e} mean {e.mean():.2e}')
