"""Debug: are in-kernel camera rays bit-identical to camera.rs rays (oracle f32)?"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from oracle import oracle as orc
from burn_raymarching_amd import render, model
sc = model.synthetic_scene(32, 5)
s = model.scene_tensors(sc)
for cam in model.ring_cameras(3):
    for S in (0, 20):
        a = render.render_diff_camera([cam], 40, 24, s, 32.0, S).cpu().numpy()
        o, d = orc.camera_rays(40, 24, *cam, precision='f32')
        b = render.render_diff_forward(torch.from_numpy(o).cuda(), torch.from_numpy(d).cuda(), s, 32.0, S).cpu().numpy()
        o2, d2 = render.create_camera_rays(40, 24, *cam)
        c = render.render_diff_forward(o2, d2, s, 32.0, S).cpu().numpy()
        print('S', S, 'cam-vs-oracle rays: n diff', (a != b).any(1).sum(), 'max', np.abs(a-b).max(),
              '| python rays vs oracle rays equal:', np.array_equal(d2.cpu().numpy(), d), np.abs(d2.cpu().numpy()-d).max())
