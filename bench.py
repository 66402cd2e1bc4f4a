#!/usr/bin/env python3
"""bench.py -- fragments/s of the repeat-fragment classification hot path on MI355X.

Workload (BASELINE.json configs[2], "cfg3"): 50M synthetic fragments of a 3 Gbp
self-comparison (SURVEY.md §8d generator), ratios (0.3, 0.3).  One step = one
rk_classify_device call: SoA inputs already resident in HBM -> group id, repeat
flag and output order in HBM (the reference's generate_fragment_groups +
generate_diagonal_func + sort_groups + repeat flag, commonFunctions.cpp:41-177).

Multi-GPU (`torchrun --nproc-per-node N bench.py --gpus N`): one process per GPU.
`value` at N>1 (default `--mode auto`): the SAME 50M-fragment set as the N=1
line (cfg3's seed-3 set, pinned by tests/golden/large_hashes.json), rank r
holding file rows [50M r / N, 50M (r+1) / N), classified by rk_classify_sharded
with RCCL all-to-alls over xGMI (xStart/10 slices, X/Y halo exchange,
cross-slice roots, gid-range member sort; DESIGN.md "Multi-GPU") -- strong
scaling.  After the timed region every rank's output share is gathered to rank
0 and the whole result's digest is checked against the reference's (`parity`).
The same run first measures
`replicas`: every rank classifies its own independent 50M set (no data-path
collective), reported beside the value under `replicas`, never as it: if the
sharded leg fails, `value` is null and the error is reported.  A gloo barrier
brackets every timed region and the max time over ranks is reported.

Rank 0 prints ONE JSON line.  Extra keys: `roofline` for the kernel with the
most device time per step (algorithmic bytes per launch / HIP-event launch time
measured inside the timed steps -- only that kernel's launches carry events
there, so the timers cost the step little; PMC HBM traffic from
profiles/traffic.json), `kernels` (every kernel, from PROFILED_STEPS further
steps with every launch timed, after the timed region),
`cpu_baseline` (1 core of this host: the reference itself,
oracle/_ref/ref_driver, on a bounded sample of the workload as the value; the
in-repo restatement on the SAME arrays the GPU classified beside it, result
compared; this host's nproc), `parity` (the timed
steps' result digest against the reference's, tests/golden/large_hashes.json),
`host_to_host_fragments_per_s` (rk_classify from host buffers, PCIe included),
`phases_ms` (per-step device time per phase).
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
    # BASELINE.json configs[4] is quoted for 8 GPUs ("streaming / HBM-spill");
    # its 1B fragments fit one MI355X's HBM too (run it with --no-cpu)
    "cfg5": dict(n=1_000_000_000, genome_len=15_000_000_000,
                 synth=dict(family_frac=0.95, copies=(100, 600)),
                 desc="cfg5: 1B fragments, 15 Gbp repeat-rich self-comparison"),
}



def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        sys.stdout.flush()  # gloo prints its connection banner on stdout: keep it off
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    return rank, world, local


def log(msg: str) -> None:
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print(f"[bench {time.strftime('%H:%M:%S')} rank {os.environ.get('RANK', '0')}] {msg}",
          file=sys.stderr, flush=True)


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


# the reference sample's size: at most this many fragments, over the genome
# scaled to keep the config's density (cfg3: 12.5M fragments over 750 Mbp,
# ~15-20 s of the reference's grouping + sorting on one core)
REF_SAMPLE_MAX = 12_500_000


def reference_sample(cfg: dict, seconds_hint: float) -> dict | None:
    """The reference itself (oracle/_ref/ref_driver, compiled from
    /root/reference/src by oracle/ref.mk) on a bounded sample of the same
    workload: the config's generator and density at min(n, 12.5M) fragments,
    timed over generate_fragment_groups + generate_diagonal_func + sort_groups
    on one core of this host."""
    from oracle import rk_oracle as ro
    if not os.path.exists(ro.REF_DRIVER):
        return None
    n = min(cfg["n"], REF_SAMPLE_MAX)
    L = cfg["genome_len"] * n // cfg["n"]
    f = rk.synth(n, L, seed=3, **cfg.get("synth", {}))
    with tempfile.TemporaryDirectory() as d:
        inp = os.path.join(d, "sample.csv")
        rk.write_input_csv(inp, f, L, L)
        del f
        p = subprocess.run([ro.REF_DRIVER, inp, "-", "0.3", "0.3"], capture_output=True,
                           text=True, timeout=max(300.0, seconds_hint * 10))
    if p.returncode != 0:
        return None
    t = json.loads(p.stderr.strip().splitlines()[-1])
    hot = t["group_s"] + t["diag_sort_s"]
    frac = f"1/{cfg['n'] // n}" if n < cfg["n"] else "all"
    return {"value": round(n / hot, 1), "unit": "fragments/s", "cores": 1, "kind": "reference",
            "sample": f"{n} fragments over {L} bp ({frac} of the config, at its density and "
                      f"generator), ratios 0.3/0.3; the reference's own code "
                      f"(oracle/_ref/ref_driver built from /root/reference/src), timed region "
                      f"generate_fragment_groups + generate_diagonal_func + sort_groups "
                      f"({hot:.2f} s; its CSV load {t['load_s']:.2f} s not counted); "
                      f"host: {host_cpu()}",
            "seconds": round(hot, 3)}


def host_cpu() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores() -> dict:
    """This host's CPUs: nproc (every online CPU) and the ones this process may use."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cpu_model": host_cpu()}


def port_same_input(cfg: dict, same_input) -> dict:
    """The in-repo restatement (oracle/rk_oracle.c, one thread) on the SAME arrays
    the GPU classified, its result compared with the GPU's."""
    from oracle import rk_oracle as ro
    f, L, gpu_digest = same_input
    t0 = time.perf_counter()
    rc, gid, rep, order, _ = ro.classify(f.x_start, f.y_start, f.length, f.strand, L, L, 0.3, 0.3)
    dt = time.perf_counter() - t0
    out = {"value": round(f.n / dt, 1), "unit": "fragments/s", "cores": 1, "kind": "port",
           "sample": f"the full {f.n}-fragment input the GPU classified (same arrays, same host), "
                     f"ratios 0.3/0.3; oracle/rk_oracle.c restatement, one thread ({dt:.2f} s)",
           "same_result_as_gpu": bool(rc == 0 and arrays_sha256(order, gid, rep) == gpu_digest)}
    ratio = port_reference_ratio(cfg)
    if ratio:
        out["port_over_reference_time"] = ratio
        out["reference_equivalent_value"] = round(f.n / dt * ratio, 1)
    return out


def cpu_baseline(cfg: dict, seconds_hint: float, same_input=None) -> dict | None:
    """CPU baseline on this host, 1 core.

    value: the REFERENCE itself on a bounded sample of the workload
    (`reference_sample`).  Beside it: the in-repo restatement on the same full
    arrays the GPU classified (`port_same_input`, result compared with the
    GPU's), the reference's full-size rate from the build container
    (`full_size`), and this host's core count."""
    sample = reference_sample(cfg, seconds_hint)
    port = port_same_input(cfg, same_input) if same_input is not None else None
    full = full_size_reference(cfg)
    out = sample if sample is not None else port
    if out is None:
        return None
    if out is sample and port is not None:
        out["port_same_input"] = port
    if sample is not None and full:
        out["sample_over_full"] = round(sample["value"] / full["value"], 2)
    if full:
        out["full_size"] = full
    node = full_size_on_node(cfg)
    if node:
        out["full_size_on_gpu_host"] = node
    out["host"] = host_cores()
    return out


def full_size_on_node(cfg: dict) -> dict | None:
    """The reference on the WHOLE cfg3 file as timed by tools/io_bench.py on a
    GPU box's host (profiles/r6_io_bench.json, committed; not this run)."""
    if cfg is not CONFIGS["cfg3"]:
        return None
    try:
        with open(os.path.join(ROOT, "profiles", "r6_io_bench.json")) as fh:
            e = json.load(fh)
        r = e["reference"]
        hot = r["group_s"] + r["diag_sort_s"]
        return {"value": round(e["fragments"] / hot, 1), "unit": "fragments/s", "cores": 1,
                "kind": "reference",
                "sample": f"the full set ({e['fragments']} fragments, the same generator and "
                          f"seed), group + diag/sort {hot:.1f} s on {e['host']['cpu_model']}; "
                          f"measured by tools/io_bench.py (profiles/r6_io_bench.json), "
                          f"not in this run"}
    except (OSError, ValueError, KeyError):
        return None


def port_reference_ratio(cfg: dict):
    """restatement time / reference time on the same full input, both measured
    in the build container (tests/golden/large_hashes.json)."""
    e = large_entry(cfg)
    if not e or "oracle_classify_s" not in e or "ref_timing" not in e:
        return None
    t = e["ref_timing"]
    return round(e["oracle_classify_s"] / (t["group_s"] + t["diag_sort_s"]), 3)


def large_entry(cfg: dict):
    name = next((k for k, v in CONFIGS.items() if v is cfg), None)
    try:
        with open(os.path.join(ROOT, "tests", "golden", "large_hashes.json")) as fh:
            return json.load(fh).get(name or "")
    except (OSError, ValueError):
        return None


def arrays_sha256(*arrs) -> str:
    import hashlib
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).view(np.uint8).data)
    return h.hexdigest()


def full_size_reference(cfg: dict) -> dict | None:
    """The reference's hot-path rate on the WHOLE config (not a sample), as pinned
    by tests/golden/make_golden_large.py (the reference binary classifying the
    full cfg3 CSV in the build container, 1 core): the sample's rate overstates
    it, since the reference's per-fragment cost grows with the set's size."""
    e = large_entry(cfg)
    t = e.get("ref_timing") if e else None
    if not t:
        return None
    hot = t["group_s"] + t["diag_sort_s"]
    return {"value": round(t["frags"] / hot, 1), "unit": "fragments/s", "cores": 1,
            "kind": "reference",
            "sample": f"the full set ({t['frags']} fragments), timed region "
                      f"generate_fragment_groups + generate_diagonal_func + sort_groups "
                      f"({hot:.1f} s), measured in the build container "
                      f"(tests/golden/large_hashes.json ref_timing), not on this host"}


def load_traffic(kernel: str, config: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (tools/pmc_run.sh -> profiles/traffic.json, or traffic_<config>.json for
    another config), only when they were measured on this run's config;
    otherwise None (not measured for this workload)."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    alt = os.path.join(ROOT, "profiles", f"traffic_{config}.json")
    if os.path.exists(alt):
        path = alt
    try:
        with open(path) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None
    if t.get("config") != config:
        return None
    return t.get("kernels", {}).get(kernel, {}).get("hbm_bytes_per_launch")


def roofline_of(kt: dict, steps: int, config: str):
    """Per-kernel HIP-event timing (inside the timed steps, on the library's
    stream) -> the `kernels` table and the roofline of the kernel with the most
    device time per step."""
    kernels = {}
    for name, k in kt.items():
        gbps = k["algo_bytes"] / (k["total_ms"] * 1e-3) / 1e9 if k["total_ms"] and k["algo_bytes"] else None
        kernels[name] = {"ms_per_step": round(k["total_ms"] / steps, 3),
                         "launches_per_step": round(k["launches"] / steps, 2),
                         "algo_GBps": round(gbps, 1) if gbps else None}
    if not kt:  # profiling off (RK_BENCH_NOPROF)
        return kernels, None
    dom = max(kt, key=lambda n: kt[n]["total_ms"])
    d = kt[dom]
    launch_ms = d["total_ms"] / max(1, d["launches"])
    bytes_per_launch = d["algo_bytes"] / max(1, d["launches"])
    achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9 if launch_ms else 0.0
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": load_traffic(dom, config), "kernel": dom,
                "algorithmic_bytes_per_launch": round(bytes_per_launch),
                "launch_ms": round(launch_ms, 4),
                "launches_per_step": round(d["launches"] / steps, 2),
                "kernel_ms_per_step": round(d["total_ms"] / steps, 3)}
    return kernels, roofline


# the record pipeline's dominant kernel (DESIGN.md kernel table): the one
# kernel whose launches carry HIP events inside the timed steps
ROOFLINE_KERNEL = "k_onesweep"
PROFILED_STEPS = 3  # steps after the timed region with every launch timed


def timed(step, args, world, ctx):
    """W untimed steps, then K timed steps between barriers + device syncs
    (phase events and the roofline kernel's launch events on; RK_BENCH_NOPROF=1
    turns them off, RK_BENCH_ALLPROF=1 times every launch there instead)."""
    for _ in range(args.warmup):
        step()
    if os.environ.get("RK_BENCH_NOPROF"):
        ctx.set_profiling(False)
    else:
        ctx.set_profiling(True, None if os.environ.get("RK_BENCH_ALLPROF") else ROOFLINE_KERNEL)
    ctx.reset_phases()
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    out = None
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    barrier(world)
    dt = time.perf_counter() - t0
    ctx.set_profiling(False)
    return out, dt


def kernel_tables(step, args, ctx, config: str):
    """`roofline` from the timed steps' launch events (read before this is
    called: ctx.kernel_timing() right after timed()) and the `kernels` table
    from PROFILED_STEPS more steps with every launch timed."""
    kt_timed = ctx.kernel_timing()
    _, roofline = roofline_of(kt_timed, args.steps, config)
    ctx.set_profiling(True)
    ctx.reset_phases()
    for _ in range(PROFILED_STEPS):
        step()
    torch.cuda.synchronize()
    ctx.set_profiling(False)
    kernels, roof_all = roofline_of(ctx.kernel_timing(), PROFILED_STEPS, config)
    if roof_all and (not roofline or roofline["kernel"] != roof_all["kernel"]):
        # another kernel dominates (e.g. the generic pipeline ran): its figures
        # come from the profiled steps
        roof_all["timed_in"] = f"{PROFILED_STEPS} profiled steps after the timed region"
        roofline = roof_all
    elif roofline:
        roofline["timed_in"] = ("the timed steps (every launch timed)" if os.environ.get("RK_BENCH_ALLPROF")
                                else "the timed steps (this kernel's launches only)")
    return kernels, roofline


def upload(f, dev):
    return (torch.from_numpy(f.x_start.view(np.int64)).to(dev),
            torch.from_numpy(f.y_start.view(np.int64)).to(dev),
            torch.from_numpy(f.length.view(np.int64)).to(dev),
            torch.from_numpy(f.strand).to(dev))


def config_seed(name: str) -> int:
    """The generator seed of a config's ONE fragment set: its number (cfg3 -> 3,
    the seed tests/golden/large_hashes.json pins for cfg3 / cfg4)."""
    return int(name[3:])


def row_block(n: int, rank: int, world: int) -> tuple[int, int]:
    """Rank r's contiguous block of file-order rows of an n-row set."""
    return n * rank // world, n * (rank + 1) // world


def gather_result(world: int, rank: int, off: int, order, gid, rep, n_total: int):
    """Every rank's share of the output (output rows [off, off + len(order)) of the
    whole result) to rank 0, which returns the whole (order, gid, rep); other
    ranks return None.  Shares must tile [0, n_total) exactly."""
    order = np.ascontiguousarray(order, dtype=np.uint32)
    gid = np.ascontiguousarray(gid, dtype=np.uint32)
    rep = np.ascontiguousarray(rep, dtype=np.uint8)
    k = len(order)
    if world == 1:
        assert off == 0 and k == n_total, (off, k, n_total)
        return order, gid, rep
    import torch.distributed as dist
    meta = torch.tensor([off, k], dtype=torch.int64)
    metas = [torch.empty(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(metas, meta)
    spans = [(int(m[0]), int(m[1])) for m in metas]
    kmax = max(1, max(c for _, c in spans))
    buf = torch.zeros(9 * kmax, dtype=torch.uint8)
    b = buf.numpy()
    b[:4 * k] = order.view(np.uint8)
    b[4 * kmax:4 * kmax + 4 * k] = gid.view(np.uint8)
    b[8 * kmax:8 * kmax + k] = rep
    bufs = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, bufs, dst=0)
    if rank != 0:
        return None
    out_o, out_g = np.empty(n_total, np.uint32), np.empty(n_total, np.uint32)
    out_r = np.empty(n_total, np.uint8)
    pos = 0
    for (o, c), t in sorted(zip(spans, bufs), key=lambda st: st[0][0]):
        assert o == pos, f"output shares do not tile: share at {o}, expected {pos}"
        a = t.numpy()
        out_o[o:o + c] = a[:4 * c].view(np.uint32)
        out_g[o:o + c] = a[4 * kmax:4 * kmax + 4 * c].view(np.uint32)
        out_r[o:o + c] = a[8 * kmax:8 * kmax + c]
        pos += c
    assert pos == n_total, (pos, n_total)
    return out_o, out_g, out_r


def bench_sharded(args, cfg, rank, world, local, dev, ctx) -> dict:
    """ONE fragment set over the ranks (strong scaling): the config's own
    single-seed set (cfg3: the 50M rows pinned by large_hashes.json), every
    rank generating it deterministically and keeping its contiguous block of
    file-order rows.  After the timed region every rank's output share goes to
    rank 0, which checks the whole result's digest against the reference's.
    cfg5 (1B rows: one whole copy per rank does not fit the host) is instead
    world independently seeded blocks of n / world rows (no digest)."""
    n_cfg, L = cfg["n"], cfg["genome_len"]
    a, b = row_block(n_cfg, rank, world)
    # the one-set route makes every rank generate the WHOLE set (~64 B per row
    # with the generator's temporaries) before keeping its block: only when
    # all ranks' copies fit half of this host's free memory
    try:
        import psutil
        free = psutil.virtual_memory().available
    except Exception:  # noqa: BLE001 -- unknown: assume it fits
        free = float("inf")
    one_set = not cfg.get("synth") and world * n_cfg * 64 <= 0.5 * free
    if one_set:
        f = rk.synth(n_cfg, L, seed=config_seed(args.config), with_ident=False)
        f = rk.Frags(f.x_start[a:b], f.y_start[a:b], f.length[a:b], f.strand[a:b])
    else:
        f = rk.synth(b - a, L, seed=rank_seed(rank), with_ident=False, **cfg.get("synth", {}))
    n = b - a
    x, y, ln, s = upload(f, dev)
    del f
    log(f"sharded: rows [{a}, {b}) of {n_cfg} uploaded")
    comm = (rk.Comm.rccl(rank, world, local) if args.comm == "rccl"
            else rk.Comm.torch_host(rank, world))
    log(f"sharded: {args.comm} comm up")

    def step():
        return rk.classify_sharded(ctx, comm, x, y, ln, s, L, L, args.len_ratio, args.pos_ratio,
                                   copy=False)

    out, dt = timed(step, args, world, ctx)
    log(f"sharded: {args.steps} timed steps in {dt:.3f} s")
    frags_total, dt_max = aggregate(world, n, dt)
    # the timed steps' result, before any further step runs
    share = rk.shard_copy(ctx, out)
    st = rk.shard_stats(ctx)
    sent = allsum(world, float(st["bytes_sent"]))
    kernels, roofline = kernel_tables(step, args, ctx, f"{args.config}-sharded-x{world}")
    comm.close()
    whole = gather_result(world, rank, out.out_offset, share.out_order, share.gid, share.repval,
                          out.n_out_total)
    log("sharded: result gathered")
    parity = None
    if rank == 0:
        digest = arrays_sha256(*whole)
        e = large_entry(cfg)
        pinned = (one_set and e is not None
                  and e.get("synth", {}).get("seed") == config_seed(args.config)
                  and e["synth"].get("n") == n_cfg and e["synth"].get("genome_len") == L
                  and e.get("len_ratio") == args.len_ratio and e.get("pos_ratio") == args.pos_ratio)
        parity = {"result_sha256": digest,
                  "matches_reference_digest": (digest == e["result_sha256"]) if pinned else None,
                  "gathered_from_ranks": world,
                  "pinned_by": ("tests/golden/large_hashes.json (the reference's output for this "
                                "input; cfg4: the restatement's, pinned to the reference at cfg3)"
                                if pinned else "no reference digest for this input")}
        del whole
    value = frags_total * args.steps / dt_max
    n_all = int(frags_total)
    return {
        "value": round(value, 1), "unit": "fragments/s", "n_gpus": world,
        "ms_per_step": round(dt_max / args.steps * 1e3, 3),
        "scaling": "strong",
        "workload": (f"ONE {n_all}-fragment set over a {L} bp genome, sharded over {world} GPUs: "
                     + (f"{args.config}'s single seed-{config_seed(args.config)} set (the "
                        f"one-GPU line's input), rank r holding file rows "
                        f"[{n_cfg} r / {world}, {n_cfg} (r+1) / {world})" if one_set else
                        f"{world} independently seeded blocks of ~{n} rows (cfg's size and "
                        f"genome; not the single-seed set of the one-GPU {args.config} run)")),
        "fragments_total": n_all, "comm": args.comm,
        "hbm_algorithmic_GBps": round(50 * value / 1e9, 3),
        "roofline": roofline, "kernels": kernels,
        "shard_rank0": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()},
        "exchange_bytes_per_step": round(sent),
        "groups": out.n_groups, "grouped_fragments": out.n_out_total,
        "parity": parity,
    }


def host_legs(ctx, x, y, ln, s, L, args) -> dict:
    """rk_classify from host buffers: `steps` calls each with pageable (numpy)
    and page-locked (pinned torch) buffers; per call the upload, device and
    download times (rk_stats h2d_ms / device_ms / d2h_ms) and the whole call."""
    n = x.shape[0]
    out = {}
    for kind in ("pageable", "pinned"):
        pin = kind == "pinned"
        cols = []
        for t in (x, y, ln, s):
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=pin)
            h.copy_(t)
            cols.append(h)
        f = rk.Frags(*[c.numpy().view(np.uint64) if c.dtype == torch.int64 else c.numpy()
                       for c in cols])
        res = [torch.empty(n, dtype=dt, pin_memory=pin).numpy() for dt in
               (torch.int32, torch.uint8, torch.int32)]
        gid, rep, order = res[0].view(np.uint32), res[1], res[2].view(np.uint32)
        ctx.classify_into(f, L, L, args.len_ratio, args.pos_ratio, gid, rep, order)  # warm-up
        acc = {"h2d_ms": 0.0, "kernels_ms": 0.0, "d2h_ms": 0.0}
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ctx.classify_into(f, L, L, args.len_ratio, args.pos_ratio, gid, rep, order)
            st = ctx.stats()
            acc["h2d_ms"] += st["h2d_ms"]
            acc["kernels_ms"] += st["device_ms"]
            acc["d2h_ms"] += st["d2h_ms"]
        dt = time.perf_counter() - t0
        out[kind] = {"fragments_per_s": round(n * args.steps / dt, 1),
                     "ms_per_call": round(dt / args.steps * 1e3, 3),
                     **{k: round(v / args.steps, 3) for k, v in acc.items()},
                     # NUMA nodes (-1: unknown / unbound): the caller's input pages,
                     # the packing threads' binding, the pinned staging slots, the GPU
                     "numa": {k: st[f"numa_{k}"] for k in ("input", "threads", "staging",
                                                           "gpu")}}
        del cols, f, res
    out["steps"] = args.steps
    out["note"] = ("host wall time per call; kernels_ms = HIP-event time of the device "
                   "pipeline inside the call; the packing threads are bound to the node of "
                   "the caller's pages (RK_IO_NUMA=0: unbound)")
    return out


def bench_single(args, cfg, rank, world, dev, ctx) -> dict:
    """rk_classify_device on this rank's own fragment set (inputs resident in HBM)."""
    n, L = cfg["n"], cfg["genome_len"]
    f = rk.synth(n, L, seed=rank_seed(rank), **cfg.get("synth", {}))  # own set per rank
    x, y, ln, s = upload(f, dev)
    gid = torch.empty(n, dtype=torch.int32, device=dev)
    rep = torch.empty(n, dtype=torch.uint8, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    # the host arrays stay for the same-input CPU baseline (rank 0, one GPU)
    keep_host = rank == 0 and world == 1 and not args.no_cpu and n <= 50_000_000
    if not keep_host:
        del f

    def step():
        return ctx.classify_device(x, y, ln, s, gid, rep, order, L, L, args.len_ratio,
                                   args.pos_ratio)

    log(f"single: {n} rows uploaded")
    (n_out, n_groups), dt = timed(step, args, world, ctx)
    log(f"single: {args.steps} timed steps in {dt:.3f} s")
    frags_total, dt_max = aggregate(world, n, dt)
    phases = ctx.phases()
    st = ctx.stats()
    kernels, roofline = kernel_tables(step, args, ctx, args.config)

    # host-to-host rate (host SoA in, host results out: rk_classify), reported
    # beside value, never as it (SURVEY.md §8d's PCIe-inclusive timed region)
    host = None
    if rank == 0 and args.config in ("cfg2", "cfg3", "cfg4"):  # cfg5: no HBM for a 2nd copy
        host = host_legs(ctx, x, y, ln, s, L, args)
    per_step = {k: v[0] / max(1, v[1]) for k, v in phases.items()}
    value = frags_total * args.steps / dt_max
    # the result of the timed steps, digested (tests/test_large_configs.py's
    # definition) and compared with the REFERENCE's result for this input where
    # tests/golden/large_hashes.json pins it (cfg3: seed 3 = rank 0's set)
    digest = arrays_sha256(order[:n_out].cpu().numpy().view(np.uint32),
                           gid[:n_out].cpu().numpy().view(np.uint32), rep[:n_out].cpu().numpy())
    e = large_entry(cfg)
    pinned = (e is not None and e.get("synth", {}).get("seed") == rank_seed(rank)
              and e["synth"].get("n") == n and e["synth"].get("genome_len") == L
              and not cfg.get("synth"))
    parity = {"result_sha256": digest,
              "matches_reference_digest": (digest == e["result_sha256"]) if pinned else None,
              "pinned_by": ("tests/golden/large_hashes.json (the reference's output for this "
                            "input, reproduced byte-exact as CSV by test_cfg3_reference_csv)"
                            if pinned else "no reference digest for this input")}
    same_input = (f, L, digest) if keep_host else None
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
                   "parallelism": (f"independent fragment sets x{world} (weak)" if world > 1
                                   else "single GPU")},
        "hbm_algorithmic_GBps": round(50 * value / 1e9, 3),  # 50 B/fragment
        "roofline": roofline,
        "phases_ms": {k: round(v, 3) for k, v in per_step.items()},
        "kernels": kernels,
        "device_ms_per_step": round(st["device_ms"], 3),
        "groups": n_groups, "grouped_fragments": n_out,
        "sweeps": {"x": st["x_sweeps"], "y": st["y_sweeps"], "jump_rounds": st["jump_rounds"]},
        "host_to_host_fragments_per_s": host["pageable"]["fragments_per_s"] if host else None,
        "host_to_host": host,
        "parity": parity,
    }
    return line, same_input


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--len-ratio", type=float, default=0.3)
    ap.add_argument("--pos-ratio", type=float, default=0.3)
    ap.add_argument("--mode", default="auto", choices=["auto", "replicas", "sharded"],
                    help="auto: N=1 the single-GPU path, N>1 one fragment set sharded over the "
                         "GPUs (independent replicas beside it; value null if the sharded leg "
                         "fails); replicas / sharded: that leg only")
    ap.add_argument("--sharded-timeout", type=float, default=240.0,
                    help="seconds the sharded leg may take before the line is printed without it")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "host"],
                    help="sharded collectives: RCCL, or gloo host callbacks")
    args = ap.parse_args()

    rank, world, local = dist_setup()
    cfg = CONFIGS[args.config]
    if os.environ.get("RK_BENCH_SAME_GPU"):  # rehearsal: every rank on device 0
        local = 0
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    ctx = rk.Context(local)

    def sharded_line(sh: dict) -> dict:
        return {"metric": METRIC, "value": sh["value"], "unit": "fragments/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": sh["ms_per_step"],
                "higher_is_better": True, "scaling": sh["scaling"], "vs_baseline": None,
                "dtype": "u64/f64",
                "data": f"synthetic (SURVEY.md §8d generator), ONE fragment set of "
                        f"{sh['fragments_total']} fragments",
                "config": {"workload": sh["workload"],
                           "fragments_per_gpu": sh["fragments_total"] // world,
                           "genome_bp": cfg["genome_len"], "len_ratio": args.len_ratio,
                           "pos_ratio": args.pos_ratio,
                           "parallelism": f"sharded x{world} ({args.comm}): xStart/10 slices"},
                "hbm_algorithmic_GBps": sh["hbm_algorithmic_GBps"],
                "fragments_total": sh["fragments_total"],
                "roofline": sh["roofline"], "parity": sh.pop("parity"), "sharded": sh}

    same_input = None
    if args.mode == "sharded":
        line = sharded_line(bench_sharded(args, cfg, rank, world, local, dev, ctx))
    else:
        line, same_input = bench_single(args, cfg, rank, world, dev, ctx)
        if world > 1 and args.mode == "auto":
            # N > 1: the value is ONE comparison sharded over the GPUs (xStart/10
            # slices, RCCL exchanges); the independent replicas measured above
            # stay beside it.  Every rank arms the same watchdog: a stuck
            # collective must not cost the line.
            import threading

            def give_up():
                if rank == 0:
                    line["replicas"] = {"value": line["value"], "ms_per_step": line["ms_per_step"]}
                    line["value"] = line["ms_per_step"] = line["roofline"] = None
                    line["sharded"] = {"error": f"timeout after {args.sharded_timeout} s"}
                    line["cpu_baseline"] = None
                    print(json.dumps(line), flush=True)
                os._exit(3)  # a stuck collective is a failure, not a clean exit
            dog = threading.Timer(args.sharded_timeout, give_up)
            dog.daemon = True
            dog.start()
            try:
                sh = bench_sharded(args, cfg, rank, world, local, dev, ctx)
            except Exception as e:  # noqa: BLE001 -- reported with a null value
                sh = {"error": repr(e)}
            dog.cancel()
            if "error" in sh:
                # the sharded leg IS the N > 1 metric: no number for it; the
                # independent replicas stay beside the null value, never as it
                replicas = {k: line[k] for k in ("value", "ms_per_step", "scaling", "roofline",
                                                 "phases_ms", "data")}
                replicas["parallelism"] = line["config"]["parallelism"]
                line["value"] = None
                line["ms_per_step"] = None
                line["hbm_algorithmic_GBps"] = None
                line["roofline"] = None
                line["config"]["parallelism"] = f"sharded x{world} ({args.comm}): FAILED"
                line["sharded"] = sh
                line["replicas"] = replicas
            else:
                replicas = {k: line[k] for k in ("value", "ms_per_step", "scaling", "roofline",
                                                 "phases_ms", "data")}
                replicas["parallelism"] = line["config"]["parallelism"]
                line = sharded_line(sh)
                line["replicas"] = replicas
    if rank != 0:
        return
    if not args.no_cpu:
        # (N > 1: rank 0's host, the reference sample alone -- the arrays of
        # the whole set are not kept for the restatement there)
        log("cpu baseline")
        line["cpu_baseline"] = cpu_baseline(
            cfg, (line["ms_per_step"] or 0.0) / 1e3 * args.steps,
            same_input if world == 1 else None)
    else:
        line["cpu_baseline"] = None
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
