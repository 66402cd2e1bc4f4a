"""Host ingress/egress of the product (FragmentsDatabase, save_all_frag_pairs,
SaverQueue) -- CPU only.  The classification fed to the egress comes from the
oracle, so these tests pin the CSV layer independently of the GPU."""
import gzip
import os
import shutil

import numpy as np
import pytest

from conftest import EDGE, GOLDEN, edge_cases
from oracle import rk_oracle as ro

import repkiller_amd as rk


def oracle_result(db, lr, pr):
    f = db.frags
    rc, gid, rep, order, ng = ro.classify(f.x_start, f.y_start, f.length, f.strand,
                                          db.len_x_hdr, db.len_y_hdr, lr, pr)
    return rc, rk.ClassifyResult(gid, rep, order, ng)


@pytest.mark.parametrize("name,case", edge_cases(), ids=[n for n, _ in edge_cases()])
def test_ingress_egress_edge(tmp_path, name, case):
    inp = os.path.join(EDGE, name + ".in.csv")
    if case["expect"] == "error:RK_E_COUNT":
        with pytest.raises(rk.RkError) as e:
            rk.FragmentsDatabase(inp)
        assert e.value.code == -3
        return
    db = rk.FragmentsDatabase(inp)
    rc, res = oracle_result(db, case["len_ratio"], case["pos_ratio"])
    if case["expect"] != "ref":
        assert rc != 0
        return
    assert rc == 0
    out = tmp_path / "out.csv"
    db.save_all_frag_pairs(str(out), res)
    with open(os.path.join(EDGE, name + ".out.csv"), "rb") as f:
        assert out.read_bytes() == f.read()


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    d = tmp_path_factory.mktemp("c10k")
    inp = d / "in.csv"
    with gzip.open(os.path.join(GOLDEN, "corpus10k.in.csv.gz"), "rb") as fi, open(inp, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    with gzip.open(os.path.join(GOLDEN, "corpus10k.out.csv.gz"), "rb") as f:
        want = f.read()
    return str(inp), want


def test_ingress_matches_generator(corpus):
    db = rk.FragmentsDatabase(corpus[0])
    f = rk.synth(10000, 1_000_000, seed=1)
    assert db.getTotalFrags() == 10000 and db.total_hdr == 10000
    assert db.len_x_hdr == 1_000_000 and db.getA() == 1 + 1_000_001 // 10
    for a, b in ((db.frags.x_start, f.x_start), (db.frags.y_start, f.y_start),
                 (db.frags.length, f.length), (db.frags.strand, f.strand)):
        assert np.array_equal(a, b)


def test_egress_corpus10k(tmp_path, corpus):
    db = rk.FragmentsDatabase(corpus[0])
    rc, res = oracle_result(db, 0.3, 0.3)
    assert rc == 0
    out = tmp_path / "out.csv"
    db.save_all_frag_pairs(str(out), res)
    assert out.read_bytes() == corpus[1]


def test_saver_queue_and_fallback(tmp_path, corpus, monkeypatch):
    db = rk.FragmentsDatabase(corpus[0])
    rc, res = oracle_result(db, 0.3, 0.3)
    monkeypatch.chdir(tmp_path)
    sq = rk.SaverQueue(db)
    sq.addRequest(str(tmp_path / "a.csv"), res)
    sq.addRequest(str(tmp_path / "no_such_dir" / "b.csv"), res)  # -> represults-1.csv
    sq.stop()
    assert (tmp_path / "a.csv").read_bytes() == corpus[1]
    assert (tmp_path / "represults-1.csv").read_bytes() == corpus[1]


def test_missing_input_is_io_error(tmp_path):
    with pytest.raises(rk.RkError) as e:
        rk.FragmentsDatabase(str(tmp_path / "nope.csv"))
    assert e.value.code == -2


def test_synth_deterministic():
    a = rk.synth(5000, 1_000_000, seed=3)
    b = rk.synth(5000, 1_000_000, seed=3)
    c = rk.synth(5000, 1_000_000, seed=4)
    assert np.array_equal(a.x_start, b.x_start) and np.array_equal(a.strand, b.strand)
    assert not np.array_equal(a.x_start, c.x_start)


@pytest.mark.parametrize("name,case", [(n, c) for n, c in edge_cases()
                                       if c["expect"] != "error:RK_E_COUNT"],
                         ids=[n for n, c in edge_cases() if c["expect"] != "error:RK_E_COUNT"])
def test_soa_cache_edge(tmp_path, name, case):
    """The binary SoA cache holds every column the parse
    produced: a database loaded from it writes the reference's output byte for
    byte (the egress prints xEnd, yEnd, score, similarity and ident from the
    cache's columns) and has the same SoA view and header values."""
    db = rk.FragmentsDatabase(os.path.join(EDGE, name + ".in.csv"))
    cache = tmp_path / "db.soa"
    db.save_soa(str(cache))
    db2 = rk.FragmentsDatabase.load_soa(str(cache))
    assert (db2.len_x_hdr, db2.len_y_hdr, db2.total_hdr) == (db.len_x_hdr, db.len_y_hdr, db.total_hdr)
    for a, b in zip((db.frags.x_start, db.frags.y_start, db.frags.length, db.frags.strand),
                    (db2.frags.x_start, db2.frags.y_start, db2.frags.length, db2.frags.strand)):
        assert np.array_equal(a, b)
    rc, res = oracle_result(db2, case["len_ratio"], case["pos_ratio"])
    if case["expect"] != "ref":
        assert rc != 0
        return
    out = tmp_path / "out.csv"
    db2.save_all_frag_pairs(str(out), res)
    with open(os.path.join(EDGE, name + ".out.csv"), "rb") as f:
        assert out.read_bytes() == f.read()


def test_soa_cache_corpus_and_damage(tmp_path, corpus):
    """corpus10k through the cache: the reference's output byte for byte; a
    truncated, extended or foreign file is refused (RK_E_ARG), a missing one is
    RK_E_IO."""
    db = rk.FragmentsDatabase(corpus[0])
    cache = tmp_path / "db.soa"
    db.save_soa(str(cache))
    db2 = rk.FragmentsDatabase.load_soa(str(cache))
    rc, res = oracle_result(db2, 0.3, 0.3)
    assert rc == 0
    out = tmp_path / "out.csv"
    db2.save_all_frag_pairs(str(out), res)
    assert out.read_bytes() == corpus[1]
    raw = cache.read_bytes()
    for bad in (raw[:-1], raw + b"\0", b"XXXXXXXX" + raw[8:], raw[:40]):
        p = tmp_path / "bad.soa"
        p.write_bytes(bad)
        with pytest.raises(rk.RkError) as e:
            rk.FragmentsDatabase.load_soa(str(p))
        assert e.value.code in (-1, -2), e.value.code
    flipped = bytearray(raw)
    flipped[60] ^= 0x01  # inside the header text: the checksum catches it
    p = tmp_path / "flip.soa"
    p.write_bytes(bytes(flipped))
    with pytest.raises(rk.RkError) as e:
        rk.FragmentsDatabase.load_soa(str(p))
    assert e.value.code == -1
    with pytest.raises(rk.RkError) as e:
        rk.FragmentsDatabase.load_soa(str(tmp_path / "nope.soa"))
    assert e.value.code == -2
