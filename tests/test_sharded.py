"""ONE fragment set classified across several ranks (rk_classify_sharded).

Parity bar: the concatenation of the ranks' output shares is bit-identical to
the single-device path on the concatenated input (itself pinned to the oracle
and the reference's fixtures, tests/test_gpu_parity.py), and to the oracle
directly for the small sets.  Ranks share the test box's one GPU and exchange
through torch.distributed gloo (rk_comm host callbacks); the RCCL comm runs the
same driver and is exercised at world size 1.

Cases cover: ordinary synthetic sets; a dense short genome with lead_in = 0,
which forces halo disagreements and the fixed-halo re-resolution on both axes;
tiny and empty inputs (ranks without rows, slices or groups); the reference's
edge fixtures; out-of-bounds inputs, where every rank must return the same
error.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import EDGE, edge_cases
from oracle import rk_oracle as ro
import shard_worker

import repkiller_amd as rk

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(world, cases, comm_kind="host", timeout=100, env=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=shard_worker.worker,
                         args=(r, world, port, cases, q, comm_kind, env))
             for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world * len(cases)):
            ci, rank, kind, payload = q.get(timeout=timeout)
            assert kind != "crash", payload
            got[(ci, rank)] = (kind, payload)
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    return got


def assemble(got, ci, world):
    parts = []
    for r in range(world):
        kind, pl = got[(ci, r)]
        assert kind == "ok", (r, pl)
        parts.append(pl)
    parts.sort(key=lambda t: t[0])
    total, ngroups = parts[0][1], parts[0][2]
    off = 0
    for p in parts:
        assert p[0] == off and p[1] == total and p[2] == ngroups
        off += p[3].shape[0]
    assert off == total
    cat = lambda i: np.concatenate([p[i] for p in parts]) if parts else np.empty(0)  # noqa: E731
    return cat(3), cat(4), cat(5), ngroups, [p[6] for p in parts]


def reference(gpu_ctx, case):
    f, lx, ly = shard_worker.load_case(case)
    return gpu_ctx.classify(f, lx, ly, case.get("lr", 0.3), case.get("pr", 0.3)), f, lx, ly


SYNTH = [
    dict(kind="synth", n=200_000, L=20_000_000, seed=21),
    dict(kind="synth", n=200_000, L=20_000_000, seed=22, lr=0.05, pr=0.05),
    dict(kind="synth", n=100_000, L=10_000_000, seed=23, ff=0.95, copies=(100, 600)),
    # cfg5's shape (repeat-rich, long bucket runs, groups of thousands) at 1M
    dict(kind="synth", n=1_000_000, L=150_000_000, seed=28, ff=0.95, copies=(100, 600)),
    # dense: ~40 entries per 100-bp bucket and strand, no lead-in -> reruns
    dict(kind="synth", n=20_000, L=60_000, seed=24, lead_in=0),
    dict(kind="synth", n=20_000, L=60_000, seed=25, lead_in=0, lr=1.5, pr=0.7),
    # a 15-Gbp genome: coordinates and in-group keys above 2^32
    dict(kind="synth", n=300_000, L=15_000_000_000, seed=29, ff=0.95, copies=(100, 600)),
    # bucket runs of 300 / 2500 entries whose LDS lists overflow at tight ratios
    dict(kind="long_runs", runs_len=300, seed=300, L=10_000_000, lr=0.05, pr=0.05),
    dict(kind="long_runs", runs_len=2500, seed=2500, L=10_000_000, lr=0.05, pr=0.05),
    dict(kind="synth", n=7, L=1_000, seed=26),
    dict(kind="synth", n=0, L=1_000, seed=27),
]


@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_matches_single_device(gpu_ctx, world):
    got = run_ranks(world, SYNTH)
    reruns = 0
    for ci, case in enumerate(SYNTH):
        order, gid, rep, ng, stats = assemble(got, ci, world)
        want, f, lx, ly = reference(gpu_ctx, case)
        assert ng == want.n_groups, case
        assert np.array_equal(order, want.out_order), case
        assert np.array_equal(gid, want.gid), case
        assert np.array_equal(rep, want.repval), case
        if f.n <= 20_000:  # the oracle directly
            rc, ogid, orep, oorder, ong = ro.classify(f.x_start, f.y_start, f.length, f.strand,
                                                      lx, ly, case.get("lr", 0.3),
                                                      case.get("pr", 0.3))
            assert rc == 0 and ong == ng
            assert np.array_equal(order, oorder) and np.array_equal(gid, ogid)
            assert np.array_equal(rep, orep)
        if case.get("lead_in") == 0:
            reruns += sum(s["x_reruns"] + s["y_reruns"] for s in stats)
    # the dense no-lead-in sets must have exercised the fixed-halo path
    assert reruns > 0


FAST = [
    dict(kind="synth", n=200_000, L=20_000_000, seed=41, repeat=2),
    dict(kind="synth", n=100_000, L=10_000_000, seed=42, ff=0.95, copies=(100, 600), repeat=2),
    dict(kind="synth", n=300_000, L=15_000_000_000, seed=43, ff=0.95, copies=(100, 600), repeat=2),
    dict(kind="long_runs", runs_len=2500, seed=2501, L=10_000_000, lr=0.05, pr=0.05, repeat=2),
    dict(kind="synth", n=7, L=1_000, seed=44, repeat=2),
    dict(kind="synth", n=0, L=1_000, seed=45, repeat=2),
]


@pytest.mark.parametrize("world", [1, 2, 4])
def test_sharded_fast_path(gpu_ctx, world):
    """The fast path (rk_shard_fast.h): exchange sizes agreed up front through
    device-assembled messages.  Each case runs twice on the same contexts: the
    first call agrees on its buffers at every exchange, the second finds every
    stage's sizes known (no agreement points).  Both are bit-identical to the
    single device; neither falls back to the careful driver on these sets; the
    second makes at most 8 host waits and 8 all-gathers at 1, 2 and 4 ranks
    (one more of each per extra cross-slice request round)."""
    got = run_ranks(world, FAST, timeout=200)
    for ci, case in enumerate(FAST):
        order, gid, rep, ng, stats = assemble(got, ci, world)
        want, _, _, _ = reference(gpu_ctx, case)
        assert ng == want.n_groups, case
        assert np.array_equal(order, want.out_order), case
        assert np.array_equal(gid, want.gid), case
        assert np.array_equal(rep, want.repval), case
        for st in stats:
            first, second = st["calls"]
            assert first["fast_path"] == 1 and second["fast_path"] == 1, st
            assert first["fast_retry"] == 0 and second["fast_retry"] == 0, (case, st)
            assert second["generic_driver"] == 0
            if world > 1:
                assert second["fast_stages"] == 7, (case, second)
            extra = max(0, second["root_rounds"] - 1)
            assert second["gathers"] <= 8 + extra, (case, second)
            assert second["host_syncs"] <= 8 + extra, (case, second)


def test_sharded_fast_vs_careful(gpu_ctx):
    """RK_SH_FAST=0 (the careful driver alone) and the fast path agree, and a
    dense no-lead-in set (halo disagreements) makes the fast path hand the call
    to the careful driver, which re-resolves."""
    cases = [SYNTH[0], SYNTH[4]]
    slow = run_ranks(2, cases, env={"RK_SH_FAST": "0"})
    fast = run_ranks(2, cases)
    for ci, case in enumerate(cases):
        a = assemble(slow, ci, 2)
        b = assemble(fast, ci, 2)
        for i in range(3):
            assert np.array_equal(a[i], b[i]), case
        assert a[3] == b[3]
        assert all(st["fast_path"] == 0 for st in a[4])
        assert all(st["fast_path"] == 1 for st in b[4])
    assert any(st["fast_retry"] for st in assemble(fast, 1, 2)[4])


def _check_vs_single_device(gpu_ctx, got, cases, world, generic):
    for ci, case in enumerate(cases):
        order, gid, rep, ng, stats = assemble(got, ci, world)
        assert all(st["generic_driver"] == int(generic) for st in stats), (case, stats)
        want, _, _, _ = reference(gpu_ctx, case)
        assert ng == want.n_groups, case
        assert np.array_equal(order, want.out_order), case
        assert np.array_equal(gid, want.gid), case
        assert np.array_equal(rep, want.repval), case


# one row of ONE rank does not pack into the 16-B record (length >= 2^24): the
# agreed flag of the record driver's first stage sends every rank to the
# generic driver together (the hand-off: control words reset, then the generic
# driver's own collectives after the record driver's first gathers)
FALLBACK = [
    dict(kind="synth", n=200_000, L=20_000_000, seed=31, long_row=199_990),  # last rank's rows
    dict(kind="synth", n=200_000, L=20_000_000, seed=32, long_row=10),       # rank 0's rows
    dict(kind="synth", n=100_000, L=10_000_000, seed=33, ff=0.95, copies=(100, 600),
         long_row=50_000),
]


def test_sharded_fallback_to_generic(gpu_ctx):
    got = run_ranks(2, FALLBACK)
    _check_vs_single_device(gpu_ctx, got, FALLBACK, 2, generic=True)


def test_sharded_generic_forced(gpu_ctx):
    """RK_SHARD_GENERIC=1: the generic driver on the SYNTH sets (every row packs)."""
    cases = [c for c in SYNTH if c.get("n", 1) <= 200_000 and c["kind"] == "synth"]
    got = run_ranks(3, cases, env={"RK_SHARD_GENERIC": "1"})
    _check_vs_single_device(gpu_ctx, got, cases, 3, generic=True)


def test_sharded_order_sort_unsplit(gpu_ctx):
    """RK_NW_SPLIT=0: the slices' processing order by four LSD passes and the
    X-chunk counts by their own kernel (the default splits the sort and counts
    in the segment kernel) -- the same result."""
    cases = [SYNTH[0], SYNTH[2], SYNTH[3]]
    got = run_ranks(2, cases, env={"RK_NW_SPLIT": "0"})
    _check_vs_single_device(gpu_ctx, got, cases, 2, generic=False)


def test_sharded_y_early_schedule(gpu_ctx):
    """RK_SH_YEARLY=1: the round-3 schedule of the slices' Y sort (its head passes
    beside the X axis on the second stream) -- the same result."""
    cases = [SYNTH[0], SYNTH[3]]
    got = run_ranks(2, cases, env={"RK_SH_YEARLY": "1"})
    _check_vs_single_device(gpu_ctx, got, cases, 2, generic=False)


def test_sharded_order_split_at_cfg3_density(gpu_ctx):
    """cfg3's density (50M rows over 3 Gbp) over 4 slices: every slice takes the
    two-stage order sort.  Its coarse keys are slice-relative, so the segment
    table covers one slice's key span (with absolute coarse keys a 1M-row slice
    would need 2^11 segments against a 2017-word table and fall back to the
    four LSD passes)."""
    cases = [dict(kind="synth", n=4_000_000, L=240_000_000, seed=34)]
    got = run_ranks(4, cases, timeout=200)
    _check_vs_single_device(gpu_ctx, got, cases, 4, generic=False)
    _, _, _, _, stats = assemble(got, 0, 4)
    assert all(st["order_split"] == 1 for st in stats), stats


def test_sharded_record_driver_used(gpu_ctx):
    """Every SYNTH set packs: the record driver classified them (not the fallback)."""
    cases = SYNTH[:2]
    got = run_ranks(2, cases)
    _check_vs_single_device(gpu_ctx, got, cases, 2, generic=False)


def _edge_cases():
    out = []
    for name, case in edge_cases():
        if case["expect"] == "error:RK_E_COUNT":
            continue  # a parse error, before classification
        out.append((name, dict(kind="csv", path=os.path.join(EDGE, name + ".in.csv"),
                               lr=case["len_ratio"], pr=case["pos_ratio"],
                               expect=case["expect"])))
    return out


ERR = {"error:RK_E_UB_BUCKET": -4, "error:RK_E_UB_CENTER": -5}


def test_sharded_edge_fixtures(gpu_ctx, tmp_path):
    named = _edge_cases()
    cases = [c for _, c in named]
    world = 2
    got = run_ranks(world, cases)
    for ci, (name, case) in enumerate(named):
        if case["expect"] != "ref":
            for r in range(world):
                kind, code = got[(ci, r)]
                assert kind == "error" and code == ERR[case["expect"]], (name, r, kind, code)
            continue
        order, gid, rep, ng, _ = assemble(got, ci, world)
        db = rk.FragmentsDatabase(case["path"])
        res = rk.ClassifyResult(gid, rep, order, ng)
        out = tmp_path / f"{name}.csv"
        db.save_all_frag_pairs(str(out), res)
        with open(os.path.join(EDGE, name + ".out.csv"), "rb") as f:
            assert out.read_bytes() == f.read(), name


@pytest.mark.parametrize("env", [None, {"RK_SH_ONE": "0"}, {"RK_SH_YEARLY": "1"}],
                         ids=["one", "records", "y-early"])
def test_sharded_world_one(gpu_ctx, tmp_path, env):
    """World size 1: the rows read once as on one device (k_nw_order_hist in
    place of the row checks, the order sort's first pass on the rows; a set
    with a dropped last-bucket row or out-of-bounds rows takes the record
    route), against the single device and the reference's edge fixtures;
    RK_SH_ONE=0 forces the record route, RK_SH_YEARLY=1 the head-first Y
    schedule."""
    named = _edge_cases()
    cases = SYNTH + [c for _, c in named]
    got = run_ranks(1, cases, env=env)
    for ci, case in enumerate(SYNTH):
        order, gid, rep, ng, _ = assemble(got, ci, 1)
        want, *_ = reference(gpu_ctx, case)
        assert ng == want.n_groups, case
        assert np.array_equal(order, want.out_order) and np.array_equal(gid, want.gid), case
        assert np.array_equal(rep, want.repval), case
    for cj, (name, case) in enumerate(named):
        ci = len(SYNTH) + cj
        if case["expect"] != "ref":
            kind, code = got[(ci, 0)]
            assert kind == "error" and code == ERR[case["expect"]], (name, kind, code)
            continue
        order, gid, rep, ng, _ = assemble(got, ci, 1)
        db = rk.FragmentsDatabase(case["path"])
        out = tmp_path / f"{name}.csv"
        db.save_all_frag_pairs(str(out), rk.ClassifyResult(gid, rep, order, ng))
        with open(os.path.join(EDGE, name + ".out.csv"), "rb") as f:
            assert out.read_bytes() == f.read(), name


def test_sharded_one_rank_fails(gpu_ctx):
    """A rank that fails locally takes its peers down with it (status word in
    the driver's all-gather message): the failing rank returns its own error,
    every other rank RK_E_PEER, nobody waits, and the comm is still in step
    for the next call (the case after it succeeds bit-exactly)."""
    base = dict(kind="synth", n=50_000, L=5_000_000, seed=33)
    world = 3
    cases = [dict(base, bad_rank=1), dict(base, bad_rank=0), base]
    got = run_ranks(world, cases)
    for ci, bad in ((0, 1), (1, 0)):
        for r in range(world):
            kind, code = got[(ci, r)]
            assert kind == "error", (ci, r, kind)
            assert code == (-1 if r == bad else -11), (ci, r, code)
    order, gid, rep, ng, _ = assemble(got, 2, world)
    want, *_ = reference(gpu_ctx, base)
    assert ng == want.n_groups and np.array_equal(order, want.out_order)
    assert np.array_equal(gid, want.gid) and np.array_equal(rep, want.repval)


def test_sharded_fault_before_response_exchange(gpu_ctx):
    """A rank that fails between the cross-slice root requests and the response
    all-to-all (its response buffers are sized by skewed counts) must not leave
    its peers inside the all-to-all: the response exchange has its own
    agreement point, so the failing rank returns RK_E_NOMEM, the others
    RK_E_PEER, and the next call on the same comm is bit-exact."""
    base = dict(kind="synth", n=200_000, L=20_000_000, seed=34)
    world = 3
    cases = [dict(base, fault_rank=2, fault="k_respond"), base]
    got = run_ranks(world, cases)
    for r in range(world):
        kind, code = got[(0, r)]
        assert kind == "error", (r, kind, code)
        assert code == (-6 if r == 2 else -11), (r, code)
    order, gid, rep, ng, stats = assemble(got, 1, world)
    assert sum(s["root_rounds"] for s in stats) > 0  # the response exchange ran
    want, *_ = reference(gpu_ctx, base)
    assert ng == want.n_groups and np.array_equal(order, want.out_order)
    assert np.array_equal(gid, want.gid) and np.array_equal(rep, want.repval)


def test_sharded_rccl_single_rank(gpu_ctx):
    cases = [dict(kind="synth", n=100_000, L=10_000_000, seed=31)]
    got = run_ranks(1, cases, comm_kind="rccl")
    order, gid, rep, ng, _ = assemble(got, 0, 1)
    want, *_ = reference(gpu_ctx, cases[0])
    assert ng == want.n_groups
    assert np.array_equal(order, want.out_order) and np.array_equal(gid, want.gid)
    assert np.array_equal(rep, want.repval)


def test_cli_sharded_threads(tmp_path):
    """rk_repkiller --gpus P: one fragment set over P ranks (one thread each,
    in-process device-copy comm, all ranks on the test box's one GPU), CSV in,
    CSV out, byte-identical to the reference's output; several ratio pairs."""
    import gzip
    import shutil
    import subprocess
    from conftest import GOLDEN
    inp, out = tmp_path / "in.csv", tmp_path / "out.csv"
    with gzip.open(os.path.join(GOLDEN, "corpus10k.in.csv.gz"), "rb") as fi, open(inp, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    with gzip.open(os.path.join(GOLDEN, "corpus10k.out.csv.gz"), "rb") as f:
        want = f.read()
    for gpus in (2, 3, 5, 8):
        p = subprocess.run([rk.CLI_PATH, "--gpus", str(gpus), "--same-device", str(inp), str(out),
                            "0.05", "0.05", "0.3", "0.3"], capture_output=True, text=True,
                           timeout=300)
        assert p.returncode == 0, p.stderr
        assert out.read_bytes() == want, gpus  # last pair wins (E10)
    # a larger synthetic set against the single-GPU CLI
    f = rk.synth(300_000, 30_000_000, seed=51)
    big = tmp_path / "big.csv"
    rk.write_input_csv(str(big), f, 30_000_000, 30_000_000)
    one, four = tmp_path / "one.csv", tmp_path / "four.csv"
    for args, dst in (([], one), (["--gpus", "4", "--same-device"], four)):
        p = subprocess.run([rk.CLI_PATH, *args, str(big), str(dst), "0.3", "0.3"],
                           capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr
    assert one.read_bytes() == four.read_bytes()
