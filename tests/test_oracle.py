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


def sort_cases():
    rng = np.random.default_rng(7)
    cases = [np.array([], np.uint64), np.array([5], np.uint64)]
    for n in (2, 3, 16, 17, 18, 31, 64, 100, 257, 1000, 5000):
        cases.append(rng.integers(0, 4, n).astype(np.uint64))        # heavy ties
        cases.append(rng.integers(0, 1 << 40, n).astype(np.uint64))  # distinct
    cases.append(np.zeros(300, np.uint64))
    cases.append(np.arange(400, dtype=np.uint64)[::-1].copy())
    # median-of-3 killer (Musser) to drive the heapsort fallback
    k = 512
    a = np.zeros(k, np.uint64)
    for i in range(k // 2):
        a[2 * i] = i + 1
        a[2 * i + 1] = k // 2 + i + 1
    cases.append(a)
    return cases


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
