"""Latency of the bench step's one collective on this box: dist.all_reduce(sum) of the packed
[gradient | loss] (7M+5 fp32) over RCCL with ONE rank (the only RCCL world a one-GPU box has).
This is the launch + kernel floor of the call, a lower bound for the 8-rank xGMI all-reduce that
DESIGN.md §7's predicted scaling curve adds on top of it; the events sit on the compute stream
around the call exactly as bench.py's `ranks.allreduce_ms_per_step` does.

    python tools/allreduce_probe.py [--spheres 256 1024 4096] [--iters 200]
"""
import argparse
import json
import os
import socket

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spheres", type=int, nargs="+", default=[64, 256, 1024, 4096])
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    out = {}
    for m in args.spheres:
        buf = torch.zeros(7 * m + 5, device="cuda")
        for _ in range(20):
            dist.all_reduce(buf)
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.iters)]
        for a, b in evs:
            a.record()
            dist.all_reduce(buf)
            b.record()
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in evs)
        out[str(m)] = {"bytes": 4 * (7 * m + 5), "median_us": round(1e3 * ms[len(ms) // 2], 2),
                       "p10_us": round(1e3 * ms[len(ms) // 10], 2), "p90_us": round(1e3 * ms[9 * len(ms) // 10], 2)}
    print(json.dumps({"world": 1, "backend": "nccl (RCCL)", "allreduce": out}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
