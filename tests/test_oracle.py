"""The CPU restatement (oracle/) against the reference's own outputs (tests/golden/).

Pins the oracle before anything is compared with it: every edge fixture, the
10k corpus and the libstdc++ std::sort restatement (against std::sort itself,
compiled here by g++).  CPU only.
"""
import gzip
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import EDGE, GOLDEN, ROOT, edge_cases
from oracle import rk_oracle as ro
from sort_cases import heap_fallbacks, mcilroy_killer, sort_cases


@pytest.mark.parametrize("name,case", edge_cases(), ids=[n for n, _ in edge_cases()])
def test_oracle_edge_fixture(tmp_path, name, case):
    out = tmp_path / "out.csv"
    rc, err = ro.run_cli(ro.CLI, os.path.join(EDGE, name + ".in.csv"), str(out),
                         case["len_ratio"], case["pos_ratio"])
    if case["expect"] == "ref":
        assert rc == 0, err
        with open(os.path.join(EDGE, name + ".out.csv"), "rb") as f:
            assert out.read_bytes() == f.read()
    else:
        assert rc != 0


def test_oracle_corpus10k(tmp_path):
    inp, out = tmp_path / "in.csv", tmp_path / "out.csv"
    with gzip.open(os.path.join(GOLDEN, "corpus10k.in.csv.gz"), "rb") as fi, open(inp, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    rc, err = ro.run_cli(ro.CLI, str(inp), str(out))
    assert rc == 0, err
    with gzip.open(os.path.join(GOLDEN, "corpus10k.out.csv.gz"), "rb") as f:
        assert out.read_bytes() == f.read()


def test_oracle_boundary_hashes(tmp_path):
    """The restatement agrees with the reference's own outputs on the deviation
    boundary set (tests/boundary_cases.py, hashes from make_golden.py --boundary)."""
    import hashlib
    import json

    import boundary_cases as bc
    import repkiller_amd as rk
    with open(os.path.join(GOLDEN, "boundary_hashes.json")) as f:
        want = json.load(f)
    inp = str(tmp_path / "in.csv")
    rk.write_input_csv(inp, bc.short_dense(rk), bc.GENOME, bc.GENOME)
    with open(inp, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == want["input_sha256"]
    for lr, pr in bc.RATIOS:
        out = tmp_path / "out.csv"
        p = subprocess.run([ro.CLI, inp, str(out), lr, pr], capture_output=True, text=True)
        assert p.returncode == 0, p.stderr
        assert hashlib.sha256(out.read_bytes()).hexdigest() == want["outputs"][f"{lr},{pr}"], (lr, pr)


HARNESS = r"""
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
struct R { uint64_t key; uint32_t tag; };
int main() {
  uint64_t n; std::vector<R> v;
  while (std::fscanf(stdin, "%lu", &n) == 1) {
    v.resize(n);
    for (uint64_t i = 0; i < n; ++i) { std::fscanf(stdin, "%lu", &v[i].key); v[i].tag = (uint32_t)i; }
    std::sort(v.begin(), v.end(), [](const R &a, const R &b) { return a.key < b.key; });
    for (auto &r : v) std::printf("%u ", r.tag);
    std::printf("\n");
  }
}
"""


def test_std_sort_restatement_matches_libstdcxx(tmp_path):
    src = tmp_path / "h.cpp"
    src.write_text(HARNESS)
    exe = tmp_path / "h"
    subprocess.run(["g++", "-O2", "-std=c++14", str(src), "-o", str(exe)], check=True)
    cases = sort_cases()
    feed = "".join(f"{len(c)} " + " ".join(str(int(x)) for x in c) + "\n" for c in cases)
    out = subprocess.run([str(exe)], input=feed, capture_output=True, text=True, check=True)
    lines = out.stdout.split("\n")
    for c, line in zip(cases, lines):
        want = np.array([int(t) for t in line.split()], np.uint32)
        got = ro.std_sort(c)
        assert np.array_equal(got, want), len(c)


def test_killer_reaches_heapsort():
    for n in (100, 512, 1000, 3000):
        assert heap_fallbacks(mcilroy_killer(n)) >= 1
