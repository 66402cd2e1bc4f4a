"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference's golden outputs.  Bit-exact on every integer output: group id per
row, repeat flag per row and the output row order (hence the CSV bytes).

Sizes: edge fixtures, the 10k corpus (byte-exact CSV), synthetic cfg1/cfg2
sets against the oracle arrays, the 1M sets against the reference's SHA-256
(tests/golden/hashes.json), and property checks at larger sizes where the
oracle would be slow.
"""
import gzip
import hashlib
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import boundary_cases as bc
from long_runs import long_run_set
from conftest import EDGE, GOLDEN, ROOT, edge_cases
from oracle import rk_oracle as ro

import repkiller_amd as rk

pytestmark = pytest.mark.gpu

ERR = {"error:RK_E_UB_BUCKET": -4, "error:RK_E_UB_CENTER": -5, "error:RK_E_COUNT": -3}


def gpu_vs_oracle(ctx, f, lx, ly, lr=0.3, pr=0.3):
    got = ctx.classify(f, lx, ly, lr, pr)
    rc, gid, rep, order, ng = ro.classify(f.x_start, f.y_start, f.length, f.strand, lx, ly, lr, pr)
    assert rc == 0
    assert got.n_groups == ng
    assert np.array_equal(got.out_order, order)
    assert np.array_equal(got.gid, gid)
    assert np.array_equal(got.repval, rep)
    return got


@pytest.mark.parametrize("name,case", edge_cases(), ids=[n for n, _ in edge_cases()])
def test_edge_fixture(pctx, tmp_path, name, case):
    inp = os.path.join(EDGE, name + ".in.csv")
    if case["expect"] == "error:RK_E_COUNT":
        with pytest.raises(rk.RkError):
            rk.FragmentsDatabase(inp)
        return
    db = rk.FragmentsDatabase(inp)
    if case["expect"] != "ref":
        with pytest.raises(rk.RkError) as e:
            pctx.classify(db.frags, db.len_x_hdr, db.len_y_hdr, case["len_ratio"],
                             case["pos_ratio"])
        assert e.value.code == ERR[case["expect"]]
        return
    res = pctx.classify(db.frags, db.len_x_hdr, db.len_y_hdr, case["len_ratio"],
                           case["pos_ratio"])
    out = tmp_path / "out.csv"
    db.save_all_frag_pairs(str(out), res)
    with open(os.path.join(EDGE, name + ".out.csv"), "rb") as f:
        assert out.read_bytes() == f.read()


def test_corpus10k_csv(pctx, tmp_path):
    inp, out = tmp_path / "in.csv", tmp_path / "out.csv"
    with gzip.open(os.path.join(GOLDEN, "corpus10k.in.csv.gz"), "rb") as fi, open(inp, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    db = rk.FragmentsDatabase(str(inp))
    res = pctx.classify(db.frags, db.len_x_hdr, db.len_y_hdr)
    db.save_all_frag_pairs(str(out), res)
    with gzip.open(os.path.join(GOLDEN, "corpus10k.out.csv.gz"), "rb") as f:
        assert out.read_bytes() == f.read()


@pytest.mark.parametrize("seed", [1, 11, 12])
@pytest.mark.parametrize("lr,pr", [(0.3, 0.3), (0.05, 0.05), (1.5, 0.7), (0.3, 2.0)])
def test_cfg1_vs_oracle(pctx, seed, lr, pr):
    f = rk.synth(10000, 1_000_000, seed=seed)
    gpu_vs_oracle(pctx, f, 1_000_000, 1_000_000, lr, pr)


@pytest.mark.parametrize("n,L,kw", [
    (200_000, 10_000_000, {}),
    (200_000, 10_000_000, dict(family_frac=0.95, copies=(100, 600))),
    (50_000, 200_000, dict(family_frac=0.95, copies=(100, 600))),  # very dense buckets
    (30_000, 100_000, {}),  # upward probes active over the first 1% (c < max_index)
])
def test_synthetic_vs_oracle(pctx, n, L, kw):
    f = rk.synth(n, L, seed=21, **kw)
    gpu_vs_oracle(pctx, f, L, L)


with open(os.path.join(GOLDEN, "boundary_hashes.json")) as _f:
    BOUNDARY = json.load(_f)


@pytest.mark.parametrize("runs_len", [70, 300, 2500])
@pytest.mark.parametrize("lr,pr", [(0.05, 0.05), (0.3, 0.3), (1.5, 0.7)])
def test_long_runs_vs_oracle(pctx, runs_len, lr, pr):
    """Bucket runs longer than 64 entries (the long-run sweep), including runs
    whose ACTIVE entries overflow its LDS lists."""
    f = long_run_set(runs_len, seed=runs_len)
    gpu_vs_oracle(pctx, f, 10_000_000, 10_000_000, lr, pr)


@pytest.mark.parametrize("lr,pr", bc.RATIOS)
def test_deviation_boundaries(pctx, tmp_path, lr, pr):
    """sl == 0 / sp == 0 boundaries and NaN/inf/extreme ratios: bit-exact with
    the reference's own output (hash) and with the oracle."""
    f = bc.short_dense(rk)
    inp = str(tmp_path / "in.csv")
    rk.write_input_csv(inp, f, bc.GENOME, bc.GENOME)
    db = rk.FragmentsDatabase(inp)
    res = pctx.classify(db.frags, db.len_x_hdr, db.len_y_hdr, float(lr), float(pr))
    assert sha256_csv(db, res, str(tmp_path / "out.csv")) == BOUNDARY["outputs"][f"{lr},{pr}"]
    gpu_vs_oracle(pctx, f, bc.GENOME, bc.GENOME, float(lr), float(pr))


def test_wide_lengths_generic_sweep(gpu_ctx):
    """Lengths >= 2^31 switch the occupancy sweep to its 64-bit kernel."""
    f = rk.synth(20_000, 1_000_000, seed=41)
    rng = np.random.default_rng(41)
    k = 40
    wide = rk.Frags(rng.integers(1, 1_000_000, k).astype(np.uint64),
                    rng.integers(1, 1_000_000, k).astype(np.uint64),
                    (np.uint64(2**31) + rng.integers(0, 3, k).astype(np.uint64) * np.uint64(7)),
                    np.full(k, ord('f'), np.uint8))
    g = rk.Frags(np.concatenate([f.x_start, wide.x_start]), np.concatenate([f.y_start, wide.y_start]),
                 np.concatenate([f.length, wide.length]), np.concatenate([f.strand, wide.strand]))
    gpu_vs_oracle(gpu_ctx, g, 5_000_000_000, 5_000_000_000)


@pytest.mark.parametrize("lr,pr", [(0.05, 0.05), (0.3, 0.3)])
def test_wide_lengths_long_runs(gpu_ctx, lr, pr):
    """The 64-bit sweep on bucket runs of 2500 entries (its long-run walk,
    k_sweep_wave): the long-run set plus a few lengths >= 2^31."""
    f = long_run_set(2500, seed=77)
    k = 8
    rng = np.random.default_rng(77)
    g = rk.Frags(np.concatenate([f.x_start, rng.integers(1, 1_000_000, k).astype(np.uint64)]),
                 np.concatenate([f.y_start, rng.integers(1, 1_000_000, k).astype(np.uint64)]),
                 np.concatenate([f.length, np.full(k, 2**31 + 5, np.uint64)]),
                 np.concatenate([f.strand, np.full(k, ord('r'), np.uint8)]))
    gpu_vs_oracle(gpu_ctx, g, 5_000_000_000, 5_000_000_000, lr, pr)


def test_empty_and_tiny(pctx):
    f = rk.Frags(np.zeros(0, np.uint64), np.zeros(0, np.uint64), np.zeros(0, np.uint64),
                 np.zeros(0, np.uint8))
    r = pctx.classify(f, 1000, 1000)
    assert r.n_groups == 0 and r.out_order.size == 0
    f = rk.Frags(np.array([10], np.uint64), np.array([20], np.uint64), np.array([30], np.uint64),
                 np.array([ord('f')], np.uint8))
    gpu_vs_oracle(pctx, f, 1000, 1000)


def sha256_csv(db, res, path):
    db.save_all_frag_pairs(path, res)
    h = hashlib.sha256()
    with open(path, "rb") as fh:
        for blk in iter(lambda: fh.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


with open(os.path.join(GOLDEN, "hashes.json")) as _f:
    HASHES = json.load(_f)


@pytest.mark.parametrize("key", sorted(HASHES))
def test_1M_reference_hash(pctx, tmp_path, key):
    h = HASHES[key]
    kw = dict(h["synth"])
    if "copies" in kw:
        kw["copies"] = tuple(kw["copies"])
    f = rk.synth(**kw)
    L = kw["genome_len"]
    inp = str(tmp_path / "in.csv")
    rk.write_input_csv(inp, f, L, L)
    with open(inp, "rb") as fh:
        assert hashlib.sha256(fh.read()).hexdigest() == h["input_sha256"]
    db = rk.FragmentsDatabase(inp)
    res = pctx.classify(db.frags, db.len_x_hdr, db.len_y_hdr, h["len_ratio"], h["pos_ratio"])
    assert sha256_csv(db, res, str(tmp_path / "out.csv")) == h["output_sha256"]


def test_classify_device_torch(gpu_ctx):
    import torch
    f = rk.synth(100_000, 5_000_000, seed=7)
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(f.x_start.view(np.int64)).to(dev)
    y = torch.from_numpy(f.y_start.view(np.int64)).to(dev)
    ln = torch.from_numpy(f.length.view(np.int64)).to(dev)
    s = torch.from_numpy(f.strand).to(dev)
    gid = torch.empty(f.n, dtype=torch.int32, device=dev)
    rep = torch.empty(f.n, dtype=torch.uint8, device=dev)
    order = torch.empty(f.n, dtype=torch.int32, device=dev)
    n_out, ng = gpu_ctx.classify_device(x, y, ln, s, gid, rep, order, 5_000_000, 5_000_000)
    rc, g2, r2, o2, ng2 = ro.classify(f.x_start, f.y_start, f.length, f.strand, 5_000_000,
                                      5_000_000)
    assert ng == ng2 and n_out == o2.size
    assert np.array_equal(gid[:n_out].cpu().numpy().view(np.uint32), g2)
    assert np.array_equal(rep[:n_out].cpu().numpy(), r2)
    assert np.array_equal(order[:n_out].cpu().numpy().view(np.uint32), o2)


def test_repeat_calls_same_context(pctx):
    """Workspace reuse across sizes must not leak state between calls."""
    a = rk.synth(20_000, 2_000_000, seed=31)
    b = rk.synth(3_000, 300_000, seed=32)
    r1 = gpu_vs_oracle(pctx, a, 2_000_000, 2_000_000)
    gpu_vs_oracle(pctx, b, 300_000, 300_000)
    r3 = pctx.classify(a, 2_000_000, 2_000_000)
    assert np.array_equal(r1.out_order, r3.out_order)


PAIRS = [(0.3, 0.3), (0.05, 0.05), (1.5, 0.7), (0.3, 2.0), (float("nan"), 0.3), (0.3, 0.3)]


@pytest.mark.parametrize("n,L,kw", [
    (200_000, 10_000_000, {}),
    (50_000, 200_000, dict(family_frac=0.95, copies=(100, 600))),
])
def test_classify_pairs_vs_oracle(pctx, n, L, kw):
    """rk_classify_pairs: the shared prefix is built once and every pair's
    result equals the oracle's for that pair alone (repkiller.cpp:60-72)."""
    f = rk.synth(n, L, seed=23, **kw)
    got = pctx.classify_pairs(f, L, L, PAIRS)
    assert len(got) == len(PAIRS)
    for (lr, pr), r in zip(PAIRS, got):
        rc, gid, rep, order, ng = ro.classify(f.x_start, f.y_start, f.length, f.strand, L, L,
                                              lr, pr)
        assert rc == 0 and r.n_groups == ng, (lr, pr)
        assert np.array_equal(r.out_order, order), (lr, pr)
        assert np.array_equal(r.gid, gid), (lr, pr)
        assert np.array_equal(r.repval, rep), (lr, pr)


def test_classify_pairs_wide_and_errors(gpu_ctx):
    """Pairs over the 64-bit sweep path; invalid pair lists are rejected whole."""
    f = rk.synth(20_000, 1_000_000, seed=43)
    f.length[:25] += np.uint64(2**31)
    L = 5_000_000_000
    pairs = [(0.3, 0.3), (2.0, 0.1), (0.01, 3.0)]
    got = gpu_ctx.classify_pairs(f, L, L, pairs)
    for (lr, pr), r in zip(pairs, got):
        want = gpu_ctx.classify(f, L, L, lr, pr)
        assert r.n_groups == want.n_groups
        assert np.array_equal(r.out_order, want.out_order)
        assert np.array_equal(r.repval, want.repval)
    gpu_vs_oracle(gpu_ctx, f, L, L, 2.0, 0.1)
    with pytest.raises(rk.RkError):
        gpu_ctx.classify_pairs(f, L, L, [(0.3, 0.3), (0.0, 0.3)])
    with pytest.raises(rk.RkError):
        gpu_ctx.classify_pairs(f, L, L, [])
    e = rk.Frags(np.zeros(0, np.uint64), np.zeros(0, np.uint64), np.zeros(0, np.uint64),
                 np.zeros(0, np.uint8))
    assert [r.n_groups for r in gpu_ctx.classify_pairs(e, 100, 100, pairs)] == [0, 0, 0]


def test_cli_matches_reference(tmp_path):
    """rk_repkiller (C++ host driver) end to end: CSV in, CSV out, byte-exact."""
    inp, out = tmp_path / "in.csv", tmp_path / "out.csv"
    with gzip.open(os.path.join(GOLDEN, "corpus10k.in.csv.gz"), "rb") as fi, open(inp, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    p = subprocess.run([rk.CLI_PATH, str(inp), str(out), "0.05", "0.05", "0.3", "0.3"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    with gzip.open(os.path.join(GOLDEN, "corpus10k.out.csv.gz"), "rb") as f:
        assert out.read_bytes() == f.read()  # last pair wins (E10)
    p = subprocess.run([rk.CLI_PATH, str(inp), str(out), "0.3"], capture_output=True, text=True)
    assert p.returncode == 1  # odd ratio count: usage error (E9)
    # the binary SoA cache: written after the parse, then
    # read instead of the CSV -- the same bytes out
    cache, out2 = tmp_path / "db.soa", tmp_path / "out2.csv"
    p = subprocess.run([rk.CLI_PATH, "--save-soa", str(cache), str(inp), str(out), "0.3", "0.3"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    p = subprocess.run([rk.CLI_PATH, "--soa", str(cache), str(out2), "0.3", "0.3"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    with gzip.open(os.path.join(GOLDEN, "corpus10k.out.csv.gz"), "rb") as f:
        assert out2.read_bytes() == f.read()
    p = subprocess.run([rk.CLI_PATH, "--soa", str(inp), str(out2), "0.3", "0.3"],
                       capture_output=True, text=True)
    assert p.returncode == 1  # a CSV is not a cache


def test_std_sort_segments_vs_restatement(gpu_ctx):
    """The device introsort on adversarial segments: ties, sorted/reversed runs,
    a median-of-3 killer (depth-limit heapsort), and segments past the LDS tier."""
    from sort_cases import sort_cases
    rng = np.random.default_rng(11)
    segs = [c for c in sort_cases() if c.size > 0]
    segs += [rng.integers(0, 3, n).astype(np.uint64) for n in (600, 2000, 9000)]
    segs += [rng.integers(0, 1 << 20, 20000).astype(np.uint64)]
    keys = np.concatenate(segs)
    off = np.concatenate([[0], np.cumsum([s.size for s in segs])]).astype(np.uint32)
    perm = gpu_ctx.std_sort_segments(keys, off)
    for a, b, s in zip(off[:-1], off[1:], segs):
        want = ro.std_sort(s) + a
        assert np.array_equal(perm[a:b], want), (int(a), s.size)


@pytest.mark.parametrize("wide", [False, True])
def test_std_sort_lds_tiers_vs_restatement(gpu_ctx, wide):
    """Every LDS tier (65..2048 members): 600 segments of random sizes
    over heavy ties, few / many distinct keys, sorted, reversed and organ-pipe
    runs, and median-of-3 killers whose depth-limit heapsort falls inside the
    tier -- 32-bit keys, and 64-bit ones (`wide`)."""
    from sort_cases import heap_fallbacks, mcilroy_killer
    rng = np.random.default_rng(31 + wide)
    base = np.uint64(1 << 40) if wide else np.uint64(0)
    segs = []
    for i in range(600):
        n = int(rng.integers(65, 2049))
        kind = i % 6
        if kind == 0:
            k = rng.integers(0, 3, n)
        elif kind == 1:
            k = rng.integers(0, 40, n)
        elif kind == 2:
            k = rng.integers(0, 1 << 30, n)
        elif kind == 3:
            k = np.arange(n) if rng.integers(2) else np.arange(n)[::-1]
        elif kind == 4:
            h = n // 2
            k = np.r_[np.arange(h), np.arange(n - h)[::-1]]
        else:
            k = np.sort(rng.integers(0, 8, n))[::-1]
        segs.append(np.ascontiguousarray(k, dtype=np.uint64) + base)
    killers = [mcilroy_killer(n) + base for n in (70, 130, 300, 511, 900, 2048)]
    assert all(heap_fallbacks(k) > 0 for k in killers)
    segs += killers
    keys = np.concatenate(segs)
    off = np.concatenate([[0], np.cumsum([s.size for s in segs])]).astype(np.uint32)
    perm = gpu_ctx.std_sort_segments(keys, off)
    for a, b, sg in zip(off[:-1], off[1:], segs):
        want = ro.std_sort(sg) + a
        assert np.array_equal(perm[a:b], want), (int(a), sg.size)


def test_std_sort_large_segments_vs_restatement(gpu_ctx):
    """Segments far above the LDS cap (block-partitioned top levels, then one
    wavefront per final segment): ties, sorted, reversed, organ pipe, all
    equal, wide random keys, and a median-of-3 killer whose depth-limit
    heapsort falls on a segment above the split size."""
    from sort_cases import heap_fallbacks, mcilroy_killer
    rng = np.random.default_rng(12)
    killer = mcilroy_killer(20000)
    assert heap_fallbacks(killer) > 0
    pipe = np.r_[np.arange(25000), np.arange(25000)[::-1]].astype(np.uint64)
    segs = [rng.integers(0, 4, 300_000).astype(np.uint64),
            np.arange(100_000, dtype=np.uint64), np.arange(100_000, dtype=np.uint64)[::-1].copy(),
            pipe, np.full(70_000, 7, np.uint64), killer,
            rng.integers(0, 1 << 40, 500_000).astype(np.uint64),
            rng.integers(0, 300, 2049).astype(np.uint64),  # just past the split size
            rng.integers(0, 1 << 20, 4097).astype(np.uint64)]
    keys = np.concatenate(segs)
    off = np.concatenate([[0], np.cumsum([s.size for s in segs])]).astype(np.uint32)
    perm = gpu_ctx.std_sort_segments(keys, off)
    for a, b, s in zip(off[:-1], off[1:], segs):
        want = ro.std_sort(s) + a
        assert np.array_equal(perm[a:b], want), (int(a), s.size)


def test_std_sort_block_heapsort_vs_restatement(gpu_ctx):
    """The depth-limit heapsort of large segments (one block per segment, the
    heap's top levels in LDS, the pops' descents 6 levels per round): killers
    whose heapsort segment is just above the block threshold, straddles the
    LDS-resident levels or spans 17 levels, over all-equal, heavily tied and
    distinct keys, 32- and 64-bit (all-equal segments take the spine-ring
    path, `wave_sort_heap_equal`)."""
    from sort_cases import heap_fallbacks, killer_with_keys
    segs = [killer_with_keys(2300, 1, 1), killer_with_keys(2300, 3, 2),
            killer_with_keys(8400, 3, 3), killer_with_keys(8400, 1 << 40, 4),
            killer_with_keys(20000, 5, 5, base=1 << 40), killer_with_keys(70000, 1 << 20, 6),
            # all-equal heap segments (the lane-ring path) of odd and even length
            killer_with_keys(2301, 1, 7), killer_with_keys(33000, 1, 8),
            killer_with_keys(33001, 1, 9, base=1 << 40), killer_with_keys(65601, 1, 10)]
    for s in segs:
        assert heap_fallbacks(s) > 0
    keys = np.concatenate(segs)
    off = np.concatenate([[0], np.cumsum([s.size for s in segs])]).astype(np.uint32)
    perm = gpu_ctx.std_sort_segments(keys, off)
    for a, b, s in zip(off[:-1], off[1:], segs):
        want = ro.std_sort(s) + a
        assert np.array_equal(perm[a:b], want), (int(a), s.size)


def test_std_sort_rank_heap_vs_restatement(gpu_ctx):
    """Heap segments with a few distinct keys take the rank path (ranks-only
    pops, then every output position traced back through the pops that wrote
    its nodes): 2, 3 and 16 distinct keys (RANK_MAX), a heap beyond the
    160K-node LDS part (the deeper ranks in global memory), and 17 keys (the
    general pops again) -- against the restated std::sort."""
    from sort_cases import killer_with_keys
    segs = [killer_with_keys(30000, 2, 21), killer_with_keys(30001, 3, 22),
            killer_with_keys(12000, 16, 23, base=1 << 40), killer_with_keys(12000, 17, 24),
            killer_with_keys(400_000, 3, 25)]
    keys = np.concatenate(segs)
    off = np.concatenate([[0], np.cumsum([s.size for s in segs])]).astype(np.uint32)
    perm = gpu_ctx.std_sort_segments(keys, off)
    for a, b, s in zip(off[:-1], off[1:], segs):
        want = ro.std_sort(s) + a
        assert np.array_equal(perm[a:b], want), (int(a), s.size)


def test_std_sort_pipe_heap_packings_vs_restatement(gpu_ctx):
    """The pipelined rank pops (k_heap_pipe_pops) with the heap's ranks packed
    into LDS: 1 bit a node (2 keys, 1.2M nodes), 4 bits (16 keys, 250K), and
    heaps too large for LDS at their packing, whose bottom level stays in
    global memory (pipe_pops_tail): 3 keys at 700K (2 bits, 19 levels in LDS)
    and 16 keys at 400K (4 bits, 18 levels) -- against the restated
    std::sort."""
    from sort_cases import killer_with_keys
    segs = [killer_with_keys(1_200_000, 2, 27), killer_with_keys(250_000, 16, 28, base=1 << 40),
            killer_with_keys(700_000, 3, 29), killer_with_keys(400_000, 16, 30)]
    keys = np.concatenate(segs)
    off = np.concatenate([[0], np.cumsum([s.size for s in segs])]).astype(np.uint32)
    perm = gpu_ctx.std_sort_segments(keys, off)
    for a, b, s in zip(off[:-1], off[1:], segs):
        want = ro.std_sort(s) + a
        assert np.array_equal(perm[a:b], want), (int(a), s.size)


def test_killer_group_heap_segment_vs_oracle(gpu_ctx):
    """A group whose in-group sort keys (|yStart - diag|, commonFunctions.cpp:
    148-159) are a median-of-3 killer with 3 keys on its never-compared items:
    copies of one X fragment (each hits the first on X) at yStart = Y0 + key,
    then one more fragment of the same xStart bucket (another length: a group
    of its own) at Y0, last in the file, which sets the bucket's diagonal to
    Y0 (commonFunctions.cpp:161-177).  The record pipeline's group sort reaches
    libstdc++'s depth-limit heapsort on the group (the rank path), its count
    coming back with the call's final status word; the result against the
    oracle."""
    from sort_cases import heap_fallbacks, killer_with_keys
    k = killer_with_keys(20000, 3, 31)
    assert heap_fallbacks(k) > 0
    n, y0 = k.size, 1_000_000
    f = rk.Frags(np.full(n + 1, 5000, np.uint64), np.r_[y0 + k, y0].astype(np.uint64),
                 np.r_[np.full(n, 200), 5000].astype(np.uint64),
                 np.full(n + 1, ord('f'), np.uint8))
    got = gpu_vs_oracle(gpu_ctx, f, 2_000_000, 2_000_000)
    assert got.n_groups == 2
    # the same set twice in one call (two ratio pairs share the scratch: each
    # pair reads its heap count back on its own)
    pairs = gpu_ctx.classify_pairs(f, 2_000_000, 2_000_000, [(0.3, 0.3), (0.3, 0.3)])
    for r in pairs:
        assert np.array_equal(r.out_order, got.out_order) and np.array_equal(r.gid, got.gid)


_RICH_SCRIPT = r"""
import hashlib, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import repkiller_amd as rk
f = rk.synth(400_000, 40_000_000, seed=47, family_frac=0.95, copies=(100, 600))
ctx = rk.Context(0)
r = ctx.classify(f, 40_000_000, 40_000_000)
h = hashlib.sha256()
for a in (r.out_order, r.gid, r.repval):
    h.update(np.ascontiguousarray(a).tobytes())
print(h.hexdigest(), r.n_groups, ctx.stats()["sweep_repeats"])
"""


@pytest.mark.parametrize("env", ["RK_SPLIT_DYN=0", "RK_SPLIT_BIG=4096", "RK_SEG_WAVES=64",
                                 "RK_LONG_GRID=16", "RK_GS_WAVES_MUL=1", "RK_SWEEP_BLIND=1",
                                 "RK_SPLIT_Q=0", "RK_SPLIT_GRID=256"])
def test_schedule_switches_repeat_rich(gpu_ctx, env):
    """The grid and claiming switches of phase A (groups above 2048 members:
    dynamic claiming, its first pass' size), phase B's grid and the long-run
    walk's grid, on a repeat-rich set (cfg5's shape: groups of thousands of
    members, bucket runs of hundreds of entries) -- bit-identical to the
    default schedule; RK_SPLIT_Q=0 partitions phase A's segments through
    stopper lists in memory instead of the block-wide queue scan."""
    f = rk.synth(400_000, 40_000_000, seed=47, family_frac=0.95, copies=(100, 600))
    r = gpu_ctx.classify(f, 40_000_000, 40_000_000)
    h = hashlib.sha256()
    for a in (r.out_order, r.gid, r.repval):
        h.update(np.ascontiguousarray(a).tobytes())
    k, v = env.split("=")
    out = subprocess.run(["python", "-c", _RICH_SCRIPT, str(ROOT)], capture_output=True,
                         text=True, timeout=120, env={**os.environ, k: v})
    assert out.returncode == 0, out.stderr[-2000:]
    digest, ng, repeats = out.stdout.split()
    assert digest == h.hexdigest() and int(ng) == r.n_groups
    # the queued sweeps (3 an axis) finish this set; one queued sweep does not,
    # and the pair repeats the careful way with the same result
    assert gpu_ctx.stats()["sweep_repeats"] == 0
    assert int(repeats) == (1 if env == "RK_SWEEP_BLIND=1" else 0)


_KILLER_SCRIPT = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[1] + "/tests")
import repkiller_amd as rk
from sort_cases import killer_with_keys
segs = [killer_with_keys(30001, 3, 22), killer_with_keys(12000, 1, 26)]
keys = np.concatenate(segs)
off = np.concatenate([[0], np.cumsum([s.size for s in segs])]).astype(np.uint32)
ctx = rk.Context(0)
try:
    perm = ctx.std_sort_segments(keys, off)
except rk.RkError as e:
    print("error", e.code)
    sys.exit(0)
np.save(sys.argv[2], perm)
print("ok")
"""


@pytest.mark.parametrize("env", ["RK_HEAP_RANK=0", "RK_HEAP_PIPE=0", "RK_HEAP_TAIL=0",
                                 "RK_HEAP_ALLOC_CAP=4096"])
def test_heap_segment_switches(gpu_ctx, tmp_path, env):
    """RK_HEAP_RANK=0 (every depth-limit heap segment through the one-block
    pops of k_heap_segments), RK_HEAP_PIPE=0 (the rank pops one at a time,
    not pipelined) and RK_HEAP_TAIL=0 give the restated std::sort's
    permutation; with
    the heap path's buffers refused (RK_HEAP_ALLOC_CAP, as an exhausted HBM
    would) the call returns RK_E_NOMEM instead of writing through a null
    buffer."""
    from sort_cases import killer_with_keys
    segs = [killer_with_keys(30001, 3, 22), killer_with_keys(12000, 1, 26)]
    out_npy = tmp_path / "perm.npy"
    k, v = env.split("=")
    out = subprocess.run(["python", "-c", _KILLER_SCRIPT, str(ROOT), str(out_npy)],
                         capture_output=True, text=True, timeout=120, env={**os.environ, k: v})
    assert out.returncode == 0, out.stderr[-2000:]
    if k == "RK_HEAP_ALLOC_CAP":
        assert out.stdout.split() == ["error", str(-6)], out.stdout
        return
    assert out.stdout.strip() == "ok", out.stdout
    perm = np.load(out_npy)
    a = 0
    for sgm in segs:
        assert np.array_equal(perm[a:a + sgm.size], ro.std_sort(sgm) + a), sgm.size
        a += sgm.size


def test_pipeline_choice(gpu_ctx, generic_ctx):
    """The record pipeline runs on the BASELINE-shaped sets; inputs it cannot
    represent (a length >= 2^24) take the generic one with the same result."""
    f = rk.synth(20_000, 2_000_000, seed=61)
    gpu_vs_oracle(gpu_ctx, f, 2_000_000, 2_000_000)
    assert gpu_ctx.stats()["pipeline"] == 1
    gpu_vs_oracle(generic_ctx, f, 2_000_000, 2_000_000)
    assert generic_ctx.stats()["pipeline"] == 2
    g = rk.synth(20_000, 50_000_000, seed=62)
    g.length[777] = np.uint64(1 << 24)  # not a record: generic pipeline
    gpu_vs_oracle(gpu_ctx, g, 50_000_000, 50_000_000)
    assert gpu_ctx.stats()["pipeline"] == 2


def test_wire_format_and_fallback(gpu_ctx):
    """rk_classify's compact wire format (12-B rows up, output order + repeat
    flag down, gids rebuilt on the host from the flags: a new group wherever
    the flag is not 2, commonFunctions.cpp:101-115) on a set the record
    pipeline takes, and the SoA upload for rows outside the wire bounds (a
    length >= 2^24 here): both bit-exact with the oracle."""
    f = rk.synth(30_000, 3_000_000, seed=71)
    gpu_vs_oracle(gpu_ctx, f, 3_000_000, 3_000_000)
    st = gpu_ctx.stats()
    assert st["wire"] == 1 and st["pipeline"] == 1
    g = rk.synth(30_000, 60_000_000, seed=72)
    g.length[123] = np.uint64(1 << 24)  # beyond the wire's 24 length bits
    gpu_vs_oracle(gpu_ctx, g, 60_000_000, 60_000_000)
    st = gpu_ctx.stats()
    assert st["wire"] == 0 and st["pipeline"] == 2


def test_dense_x_chunks(gpu_ctx):
    """Dense X chunks (record pipeline): a chunk's rows are streamed in
    batches of 512 and its bins have no capacity limit, so even a single
    100-bp bucket of one strand holding thousands of entries stays on the
    record pipeline, bit-exact."""
    L = 30_000
    f = rk.synth(60_000, L, seed=63, family_frac=0.95, copies=(100, 600))
    gpu_vs_oracle(gpu_ctx, f, L, L)
    st = gpu_ctx.stats()
    assert st["pipeline"] == 1 and st["record_fallback"] == 0
    rng = np.random.default_rng(65)
    k = 3000  # one bucket, one strand: more entries than a chunk's list holds
    g = rk.Frags(np.concatenate([f.x_start, np.full(k, 5000, np.uint64)]),
                 np.concatenate([f.y_start, rng.integers(1, 20_000, k).astype(np.uint64)]),
                 np.concatenate([f.length, rng.integers(90, 110, k).astype(np.uint64)]),
                 np.concatenate([f.strand, np.full(k, ord("f"), np.uint8)]))
    gpu_vs_oracle(gpu_ctx, g, L, L)
    st = gpu_ctx.stats()
    assert st["pipeline"] == 1 and st["record_fallback"] == 0


def test_order_split_paths(gpu_ctx):
    """The processing order in two stages (coarse one-sweep passes, then one
    block per coarse-key segment sorting its fine bits, k_nw_order_fine): the
    segments in LDS (two fine passes here, F = 15), and segments above the LDS
    capacity (4096 rows) sorted through global memory, with one fine pass
    (test_dense_x_chunks) and with two (here): bit-exact with the oracle."""
    L = 10_000_000
    f = rk.synth(60_000, L, seed=66)
    gpu_vs_oracle(gpu_ctx, f, L, L)
    assert gpu_ctx.stats()["pipeline"] == 1
    rng = np.random.default_rng(67)
    k = 20_000  # xStart < 300 kbp: one coarse segment of ~21k rows
    g = rk.Frags(np.concatenate([f.x_start, rng.integers(1, 300_000, k).astype(np.uint64)]),
                 np.concatenate([f.y_start, rng.integers(1, L - 1000, k).astype(np.uint64)]),
                 np.concatenate([f.length, rng.integers(20, 400, k).astype(np.uint64)]),
                 np.concatenate([f.strand, rng.choice(np.array([ord("f"), ord("r")], np.uint8), k)]))
    gpu_vs_oracle(gpu_ctx, g, L, L)
    assert gpu_ctx.stats()["pipeline"] == 1


@pytest.mark.parametrize("pos", [1, 63, 65, 1000, 19_999])
def test_wide_length_detected_in_any_lane(pctx, pos):
    """A single length >= 2^31 at any row position switches to the 64-bit
    sweep (the device flag is a wave-wide ballot)."""
    f = rk.synth(20_000, 1_000_000, seed=64)
    f.length[pos] = np.uint64(2**31 + 3)
    gpu_vs_oracle(pctx, f, 5_000_000_000, 5_000_000_000)


_SWITCH_SCRIPT = r"""
import hashlib, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import repkiller_amd as rk
f = rk.synth(300_000, 18_000_000, seed=41)
ctx = rk.Context(0)
r = ctx.classify(f, 18_000_000, 18_000_000)
h = hashlib.sha256()
for a in (r.out_order, r.gid, r.repval):
    h.update(np.ascontiguousarray(a).tobytes())
print(h.hexdigest(), r.n_groups, ctx.stats()["sweep_repeats"])
"""


@pytest.mark.parametrize("env", ["RK_GS_BIG=0", "RK_GS_BIG=4", "RK_GS_REG1=0", "RK_GS_SMALL1=1",
                                 "RK_SWEEP_BLIND=1", "RK_NW_MINBITS=8",
                                 "RK_NW_SPLIT=0", "RK_GS_HALF=256", "RK_GS_HALF=2048",
                                 "RK_NW_YSPLIT=0", "RK_NW_MSPLIT=1", "RK_Y_OVERLAP=1",
                                 "RK_SWEEP_QUEUED=0", "RK_ROOTS_FUSED=0", "RK_ROOTS_STEPS=1",
                                 "RK_ROOTS_STEPS=1 RK_ROOTS_REST_STEPS=1", "RK_GS_SMALLPART=0"])
def test_schedule_switches_bit_identical(gpu_ctx, env):
    """The measurement switches only move work between streams or change the
    radix of a pass: the result must not change.  300k rows at cfg3 density
    (groups up to ~2000 members: every group-sort tier is used); the switch is
    read once per process, so the variant runs in a child process."""
    f = rk.synth(300_000, 18_000_000, seed=41)
    r = gpu_ctx.classify(f, 18_000_000, 18_000_000)
    h = hashlib.sha256()
    for a in (r.out_order, r.gid, r.repval):
        h.update(np.ascontiguousarray(a).tobytes())
    extra = dict(kv.split("=") for kv in env.split())
    out = subprocess.run(["python", "-c", _SWITCH_SCRIPT, str(ROOT)], capture_output=True,
                         text=True, timeout=120, env={**os.environ, **extra})
    assert out.returncode == 0, out.stderr[-2000:]
    digest, ng, repeats = out.stdout.split()
    assert digest == h.hexdigest() and int(ng) == r.n_groups
    # the queued sweeps (3 an axis) finish this set; one queued sweep does not,
    # and the pair repeats the careful way with the same result
    assert gpu_ctx.stats()["sweep_repeats"] == 0
    assert int(repeats) == (1 if env == "RK_SWEEP_BLIND=1" else 0)
