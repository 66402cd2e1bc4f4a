#!/usr/bin/env python3
"""bench.py -- fragments/s of the repeat-fragment classification hot path on MI355X.

Workload (BASELINE.json configs[2], "cfg3"): 50M synthetic fragments of a 3 Gbp
self-comparison (SURVEY.md §8d generator), ratios (0.3, 0.3).  One step = one
rk_classify_device call: SoA inputs already resident in HBM -> group id, repeat
flag and output order in HBM (the reference's generate_fragment_groups +
generate_diagonal_func + sort_groups + repeat flag, commonFunctions.cpp:41-177).

Multi-GPU (`torchrun --nproc-per-node N bench.py --gpus N`): one process per GPU,
each classifying its OWN independent 50M-fragment set (weak scaling, no data-path
collective -- DESIGN.md "Multi-GPU"); a gloo barrier brackets the timed region and
the max time over ranks is reported.

Rank 0 prints ONE JSON line.  Extra keys: `roofline` for the kernel with the
most device time per step (algorithmic bytes per launch / HIP-event launch time
measured inside the timed steps; PMC HBM traffic from profiles/traffic.json),
`kernels` (the same per kernel),
`cpu_baseline` (the reference built from its sources, oracle/_ref/ref_driver, on
a bounded sample, 1 core), `phases_ms` (per-step device time per phase).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (imported before the library: one shared HIP runtime)

import repkiller_amd as rk  # noqa: E402

METRIC = "fragments/sec filtered + achieved HBM GB/s, 50M-frag human self-cmp, 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec

CONFIGS = {
    "cfg1": dict(n=10_000, genome_len=1_000_000, desc="cfg1: 10k fragments, 1 Mbp x 1 Mbp"),
    "cfg2": dict(n=1_000_000, genome_len=100_000_000,
                 desc="cfg2: 1M fragments, 100 Mbp x 100 Mbp"),
    "cfg3": dict(n=50_000_000, genome_len=3_000_000_000,
                 desc="cfg3: 50M fragments, 3 Gbp human-scale self-comparison"),
    # BASELINE.json configs[3] is quoted for 8 GPUs; its 200M fragments also fit
    # one MI355X (~62 GB of HBM), so it runs here as a single-GPU stress case
    "cfg4": dict(n=200_000_000, genome_len=3_000_000_000,
                 desc="cfg4: 200M fragments, 3 Gbp x 3 Gbp"),
}



def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def allmax(world, v: float) -> float:
    if world == 1:
        return v
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allsum(world, v: float) -> float:
    if world == 1:
        return v
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def rank_seed(rank: int) -> int:
    """Each rank classifies its own independent fragment set (weak scaling)."""
    return 3 + rank


def aggregate(world: int, n_local: int, dt_local: float) -> tuple[float, float]:
    """Whole-job fragments and the slowest rank's time (the contract's max over ranks)."""
    return allsum(world, float(n_local)), allmax(world, dt_local)


def cpu_baseline(cfg: dict, seconds_hint: float) -> dict | None:
    """The reference (oracle/_ref/ref_driver, built from /root/reference/src by
    oracle/ref.mk) on a bounded sample of the same workload: the cfg3 density
    (fragments per bp) at 1/10 of the genome, so ~10-30 s of single-core work.
    Falls back to the in-repo restatement (oracle/_build/rk_oracle, "port")."""
    from oracle import rk_oracle as ro
    ref = ro.REF_DRIVER if os.path.exists(ro.REF_DRIVER) else None
    binary = ref or (ro.CLI if os.path.exists(ro.CLI) else None)
    if binary is None:
        try:
            ro.build_oracle()
            binary = ro.CLI
        except Exception:
            return None
    scale = 10 if cfg["n"] >= 10_000_000 else 1
    n, L = cfg["n"] // scale, cfg["genome_len"] // scale
    f = rk.synth(n, L, seed=3)
    with tempfile.TemporaryDirectory() as d:
        inp = os.path.join(d, "sample.csv")
        rk.write_input_csv(inp, f, L, L)
        out = "-" if ref else os.path.join(d, "out.csv")
        p = subprocess.run([binary, inp, out, "0.3", "0.3"], capture_output=True, text=True,
                           timeout=max(120.0, seconds_hint * 10))
    if p.returncode != 0:
        return None
    t = json.loads(p.stderr.strip().splitlines()[-1])
    hot = t["group_s"] + t["diag_sort_s"] if ref else t["classify_s"]
    cpu = subprocess.run(["sh", "-c", "grep -m1 'model name' /proc/cpuinfo | cut -d: -f2"],
                         capture_output=True, text=True).stdout.strip()
    return {"value": round(n / hot, 1), "unit": "fragments/s", "cores": 1,
            "kind": "reference" if ref else "port",
            "sample": f"{n} fragments over {L} bp (cfg3 density, 1/{scale} of the genome), "
                      f"ratios 0.3/0.3; timed region generate_fragment_groups + "
                      f"generate_diagonal_func + sort_groups ({hot:.2f} s); host: {cpu}"}


def load_traffic(kernel: str):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (tools/pmc_traffic.py)."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as fh:
            t = json.load(fh)
        return t.get("kernels", {}).get(kernel, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--len-ratio", type=float, default=0.3)
    ap.add_argument("--pos-ratio", type=float, default=0.3)
    args = ap.parse_args()

    rank, world, local = dist_setup()
    cfg = CONFIGS[args.config]
    n, L = cfg["n"], cfg["genome_len"]
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    ctx = rk.Context(local)

    f = rk.synth(n, L, seed=rank_seed(rank))  # independent fragment set per rank
    x = torch.from_numpy(f.x_start.view(np.int64)).to(dev)
    y = torch.from_numpy(f.y_start.view(np.int64)).to(dev)
    ln = torch.from_numpy(f.length.view(np.int64)).to(dev)
    s = torch.from_numpy(f.strand).to(dev)
    gid = torch.empty(n, dtype=torch.int32, device=dev)
    rep = torch.empty(n, dtype=torch.uint8, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    del f
    torch.cuda.synchronize()

    def step():
        return ctx.classify_device(x, y, ln, s, gid, rep, order, L, L, args.len_ratio,
                                   args.pos_ratio)

    for _ in range(args.warmup):
        step()
    ctx.set_profiling(True)
    ctx.reset_phases()
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n_out, n_groups = step()
    torch.cuda.synchronize()
    barrier(world)
    dt = time.perf_counter() - t0
    ctx.set_profiling(False)
    frags_total, dt_max = aggregate(world, n, dt)
    phases = ctx.phases()
    st = ctx.stats()

    # PCIe-inclusive rate (host buffers in and out), reported beside value, never as it
    pcie = None
    if rank == 0 and args.config != "cfg1":
        fh = rk.Frags(x.cpu().numpy().view(np.uint64), y.cpu().numpy().view(np.uint64),
                      ln.cpu().numpy().view(np.uint64), s.cpu().numpy())
        ctx.classify(fh, L, L, args.len_ratio, args.pos_ratio)
        t1 = time.perf_counter()
        ctx.classify(fh, L, L, args.len_ratio, args.pos_ratio)
        pcie = n / (time.perf_counter() - t1)

    if rank != 0:
        return
    per_step = {k: v[0] / max(1, v[1]) for k, v in phases.items()}
    # per-kernel HIP-event timing inside the timed steps (on the library's
    # stream); the roofline is reported for the kernel with the most device
    # time per step, whatever it is
    kt = ctx.kernel_timing()
    kernels = {}
    for name, k in kt.items():
        gbps = k["algo_bytes"] / (k["total_ms"] * 1e-3) / 1e9 if k["total_ms"] and k["algo_bytes"] else None
        kernels[name] = {"ms_per_step": round(k["total_ms"] / args.steps, 3),
                         "launches_per_step": round(k["launches"] / args.steps, 2),
                         "algo_GBps": round(gbps, 1) if gbps else None}
    dom = max(kt, key=lambda n: kt[n]["total_ms"])
    d = kt[dom]
    launch_ms = d["total_ms"] / max(1, d["launches"])
    bytes_per_launch = d["algo_bytes"] / max(1, d["launches"])
    achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9 if launch_ms else 0.0
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": load_traffic(dom), "kernel": dom,
                "algorithmic_bytes_per_launch": round(bytes_per_launch),
                "launch_ms": round(launch_ms, 4),
                "launches_per_step": round(d["launches"] / args.steps, 2),
                "kernel_ms_per_step": round(d["total_ms"] / args.steps, 3)}
    value = frags_total * args.steps / dt_max
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "fragments/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64/f64",
        "data": f"synthetic (SURVEY.md §8d generator, seed 3+rank, {n} fragments per GPU)",
        "config": {"workload": cfg["desc"], "fragments_per_gpu": n, "genome_bp": L,
                   "len_ratio": args.len_ratio, "pos_ratio": args.pos_ratio,
                   "parallelism": f"independent fragment sets x{world} (weak)"},
        "hbm_algorithmic_GBps": round(50 * value / 1e9, 3),  # 50 B/fragment
        "roofline": roofline,
        "phases_ms": {k: round(v, 3) for k, v in per_step.items()},
        "kernels": kernels,
        "device_ms_per_step": round(st["device_ms"], 3),
        "groups": n_groups, "grouped_fragments": n_out,
        "sweeps": {"x": st["x_sweeps"], "y": st["y_sweeps"], "jump_rounds": st["jump_rounds"]},
        "pcie_inclusive_fragments_per_s": round(pcie, 1) if pcie else None,
    }
    if not args.no_cpu and world == 1:
        line["cpu_baseline"] = cpu_baseline(cfg, dt_max)
    else:
        line["cpu_baseline"] = None
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
