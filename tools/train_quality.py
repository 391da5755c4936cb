"""Run the C++ train driver (train.rs schedule) on the reference's targets for several seeds and
report the final_1 preview's PSNR against the true scene, next to the reference's final_1.png."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    from burn_raymarching_amd import host, render
    from conftest import DANGO, GOLDEN, load_png
    from oracle import oracle as orc
    seeds = [int(x) for x in (sys.argv[1:] or range(8))]
    dev = torch.device("cuda:0")
    t = [torch.tensor(DANGO[k], device=dev) for k in ("centers", "colors", "radius")]
    truth = orc.to_png_bytes(render.render_camera([([0.0, 0.0, -2.5], [0.0, 0.0, 0.0], 50.0)], 256, 256, *t)
                             .cpu().numpy()).reshape(256, 256, 3).astype(np.float64)
    psnr = lambda a: 10 * np.log10(255.0 ** 2 / np.mean((a.astype(np.float64) - truth) ** 2))
    print(f"reference final_1.png: {psnr(load_png(os.path.join(GOLDEN, 'final_1.png'))):.2f} dB")
    vals = []
    for seed in seeds:
        with tempfile.TemporaryDirectory() as d:
            cfg = host.train_config(cameras_json=os.path.join(GOLDEN, "cameras.json"), out_dir=d, log_every=0,
                                    seed=seed)
            res, _ = host.train(cfg)
            p = psnr(load_png(os.path.join(d, "steps", "final_1.png")))
            vals.append(p)
            print(f"seed {seed}: {p:.2f} dB  M={res.num_spheres} loss={res.final_loss:.5f} "
                  f"{res.step_ms:.3f} ms/step", flush=True)
    print(f"median {np.median(vals):.2f} dB, min {min(vals):.2f}, max {max(vals):.2f}")


if __name__ == "__main__":
    main()
