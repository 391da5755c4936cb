"""Predicted strong-scaling curve of the default bench step (80 views of 512x512 per step over N
ranks), built from one-GPU measurements, so that the driver's 8-GPU SCALE run can be checked
against it:

    T(N) = max over ranks of the rank's train call  (profiles/*_shard_balance.json: the 80/N-view
                                                     slices timed on one GPU, each its own launch,
                                                     scaled to the bench's kernel time)
         + the step's work outside the train kernel (bench line at N = 1: ms_per_step - kernel ms;
                                                     the O(M) launches do not shrink with N)
         + one all-reduce of the 7M+5-float [gradient | loss] over N ranks:
             measured one-rank RCCL floor (tools/allreduce_probe.py) + a ring over xGMI modelled as
             2 (N - 1) latency-bound hops of HOP_US each (N > 1)

    value(N) = 80 * 512 * 512 / T(N) Mrays/s

    python tools/predict_scaling.py --bench profiles/r05_bench.json --balance profiles/r04b_shard_balance.json \
        --allreduce profiles/r05b_allreduce.json [--hop-us 2.5] [--slices 2=... 4=... 8=...] \
        > profiles/r05_scaling_prediction.json
With --per-call the N = 1 step is run as N calls of 80/N views (bench.py --views-per-call 80/N):
each call's launch is what one rank's launch is at N ranks, on the same (all-reduced) trajectory;
T(N) = one call's train kernel x (slowest / mean slice) + one call's share of the step's other
kernels + the modelled all-reduce.
With --as-rank every rank's share of the N-rank step is measured alone on one GPU (bench.py
--as-rank R/N: its fixed views, as at N ranks); alone, a rank trains on its own gradient and its
scene drifts from the all-reduced trajectory, so the prediction takes the efficiency of its launch
(the executed roofline fraction) and applies it to 1/N of the N = 1 step's executed work:
T(N) = kernel_1 x frac_1 / (N x frac_rank) x (slowest / mean slice) + the rank's time outside its
train kernel + the modelled all-reduce. With --slices the N-rank step is one rank's step measured on one GPU (bench.py --global-views
80/N --ring 80: the rank's views in one launch with its own record, origin, reduction and
optimizer kernels), its kernel stretched by the balance study's slowest-over-mean rank (the
one-GPU run rotates through the ring, so it times the mean rank), plus the modelled all-reduce.
"""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bench", required=True, help="the N = 1 bench line (JSON)")
    ap.add_argument("--balance", required=True, help="tools/shard_balance.py output")
    ap.add_argument("--allreduce", required=True, help="tools/allreduce_probe.py output")
    ap.add_argument("--order", default="spread")
    ap.add_argument("--slices", nargs="*", default=[],
                    help="N=file pairs (e.g. 8=profiles/r06i_slice_10.json): bench lines of one rank's step at N "
                         "ranks measured on one GPU (bench.py --global-views 80/N --ring 80); where given, T(N) uses "
                         "the measured step (its train kernel and its own small kernels) instead of the scaled slice")
    ap.add_argument("--as-rank", nargs="*", default=[],
                    help="N=glob pairs (e.g. 8='gpurun_out/r06n/rank_*_of_8.json'): bench lines of EVERY rank's "
                         "share of the N-rank step run alone on one GPU (bench.py --as-rank R/N: the rank's fixed "
                         "views, its own record / origin / reduction / optimizer kernels); T(N) = the slowest "
                         "rank's measured step + the modelled all-reduce. Takes precedence over --slices")
    ap.add_argument("--per-call", nargs="*", default=[],
                    help="N=file pairs: bench lines of the N = 1 step run as N calls of 80/N views "
                         "(bench.py --views-per-call 80/N: each call its own launch, context and cost "
                         "order, all on the N = 1 trajectory); T(N) = one call's train kernel x the "
                         "slowest-over-mean slice + one call's share of the other kernels + the "
                         "all-reduce. Takes precedence over --as-rank and --slices")
    ap.add_argument("--hop-us", type=float, default=2.5,
                    help="modelled latency of one xGMI ring hop of a few-KB message (no measurement on a "
                         "one-GPU box; an assumption, stated in the output)")
    args = ap.parse_args()
    b = json.load(open(args.bench))
    bal = json.load(open(args.balance))[args.order]
    ar = json.load(open(args.allreduce))["allreduce"]
    M = b["config"]["spheres"]
    rays = b["config"]["rays_per_step"]
    kern1 = b["roofline"]["kernel_ms_per_step"]
    outside = b["ms_per_step"] - kern1
    floor_us = ar[str(M)]["median_us"] if str(M) in ar else min(v["median_us"] for v in ar.values())
    out = {"inputs": {"bench": args.bench, "balance": args.balance, "allreduce": args.allreduce,
                      "kernel_ms_n1": kern1, "outside_ms": round(outside, 4), "allreduce_floor_us": floor_us,
                      "hop_us_assumed": args.hop_us},
           "curve": {}}
    measured = {}
    for pair in args.slices:
        n, f = pair.split("=", 1)
        measured[int(n)] = json.load(open(f))
    out["inputs"]["slices"] = {str(n): f for n, f in (p.split("=", 1) for p in args.slices)}
    percall = {}
    for pair in args.per_call:
        n, f = pair.split("=", 1)
        percall[int(n)] = json.load(open(f))
    out["inputs"]["per_call"] = {str(n): f for n, f in (p.split("=", 1) for p in args.per_call)}
    import glob
    shares = {}
    for pair in args.as_rank:
        n, pat = pair.split("=", 1)
        shares[int(n)] = [json.load(open(f)) for f in sorted(glob.glob(pat))]
    out["inputs"]["as_rank"] = {str(n): len(v) for n, v in shares.items()}
    for n in (1, 2, 4, 8):
        if n in percall and n > 1:
            # one rank's launch on the N = 1 trajectory: the step's N calls each a rank's views
            m = percall[n]
            r = m["roofline"]
            calls = n  # calls per step
            sl = bal[str(n)]["slice_ms"]
            imb = max(sl) / (sum(sl) / len(sl))
            kern = r["kernel_ms"] * imb  # per launch (= per call)
            other = (m["ms_per_step"] - r["kernel_ms_per_step"]) / calls
            ar_ms = (floor_us + 2 * (n - 1) * args.hop_us) * 1e-3
            t = kern + other + ar_ms
            out["curve"][str(n)] = {"step_ms": round(t, 4), "train_kernel_ms": round(kern, 4),
                                    "call_kernel_ms_measured": r["kernel_ms"], "call_frac_measured": r["frac"],
                                    "call_other_ms_measured": round(other, 4),
                                    "slowest_over_mean_rank": round(imb, 4), "allreduce_ms": round(ar_ms, 4),
                                    "mrays_s": round(rays / (t * 1e-3) / 1e6, 1)}
            continue
        if n in shares:
            # Every rank's share measured alone. Alone, a rank's Adam sees only its own views'
            # gradient, so its scene drifts differently from the all-reduced run's and the executed
            # work per ray differs (measured: 0.20-0.22 vs 0.35 of the canonical FLOP); what carries
            # over is the efficiency of the rank's launch shape (its executed roofline fraction).
            # The rank's train kernel at the N = 1 trajectory's work: 1/N of the N = 1 step's
            # executed FLOP at the rank's fraction, stretched by the slowest-over-mean slice of the
            # balance study; plus the rank's measured time outside its train kernel, plus the
            # all-reduce.
            lines = shares[n]
            fr = [m["roofline"]["frac"] for m in lines]
            frac_rank = sum(fr) / len(fr)
            sl = bal[str(n)]["slice_ms"]
            imb = max(sl) / (sum(sl) / len(sl))
            kern = kern1 * b["roofline"]["frac"] / (n * frac_rank) * imb
            outside_rank = max(m["ms_per_step"] - m["roofline"]["kernel_ms_per_step"] for m in lines)
            ar_ms = (floor_us + 2 * (n - 1) * args.hop_us) * 1e-3
            t = kern + outside_rank + ar_ms
            out["curve"][str(n)] = {"step_ms": round(t, 4), "train_kernel_ms": round(kern, 4),
                                    "rank_frac_measured": [round(x, 4) for x in fr],
                                    "rank_executed_frac_measured": [m["roofline"]["executed_frac"] for m in lines],
                                    "rank_outside_ms_measured": round(outside_rank, 4),
                                    "slowest_over_mean_rank": round(imb, 4), "allreduce_ms": round(ar_ms, 4),
                                    "ranks_measured": len(lines), "mrays_s": round(rays / (t * 1e-3) / 1e6, 1)}
            continue
        if n in measured:  # one rank's whole step measured on one GPU, plus the all-reduce
            m = measured[n]
            # the one-GPU run rotates through the ring, so it times the mean rank's slice; the step
            # waits for the slowest rank: the balance study's max / mean of the N slices adds that
            sl = bal[str(n)]["slice_ms"]
            imb = max(sl) / (sum(sl) / len(sl))
            kern = m["roofline"]["kernel_ms_per_step"]
            ar_ms = (floor_us + 2 * (n - 1) * args.hop_us) * 1e-3
            t = m["ms_per_step"] + kern * (imb - 1) + ar_ms
            out["curve"][str(n)] = {"step_ms": round(t, 4), "train_kernel_ms": round(kern * imb, 4),
                                    "slice_step_ms_measured": m["ms_per_step"], "slice_kernel_ms_measured": kern,
                                    "slowest_over_mean_rank": round(imb, 4), "allreduce_ms": round(ar_ms, 4),
                                    "mrays_s": round(rays / (t * 1e-3) / 1e6, 1)}
            continue
        if n > 1 and str(n) not in bal:  # no measurement for this N
            continue
        slice_ms = kern1 if n == 1 else max(bal[str(n)]["slice_ms"])
        # the balance study timed each rank's slice as its own launch (as the rank runs it), on a
        # scene earlier in training than the bench's timed steps: its slices are scaled by the
        # bench's kernel time over the study's two-slice total (the same 80 views)
        if n > 1:
            slice_ms *= kern1 / sum(bal["2"]["slice_ms"])
        ar_ms = 0.0 if n == 1 else (floor_us + 2 * (n - 1) * args.hop_us) * 1e-3
        t = slice_ms + outside + ar_ms
        out["curve"][str(n)] = {"step_ms": round(t, 4), "train_kernel_ms": round(slice_ms, 4),
                                "allreduce_ms": round(ar_ms, 4), "mrays_s": round(rays / (t * 1e-3) / 1e6, 1)}
    v1 = out["curve"]["1"]["mrays_s"]
    for n in (k for k in ("2", "4", "8") if k in out["curve"]):
        out["curve"][n]["efficiency"] = round(out["curve"][n]["mrays_s"] / (int(n) * v1), 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
