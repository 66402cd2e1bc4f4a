"""The reference-side binding (integration/rk_reference_shim.cpp, shown in
INTEGRATION.md) against the reference's REAL headers.

CPU: the shim and its driver compile and link against /root/reference/src
(FragmentsDatabase.h, structs.h, commonFunctions.h) and librepkiller_amd.so
(oracle/shim.mk) -- a drift in the conventions the shim relies on
(FragmentsDatabase::begin/end, sequence_manager::get_sequence_by_label(..).len,
FGList / FragsGroup, execWithParams' call sequence, repkiller.cpp:80-97,
structs.h:79-91) breaks this build.  Skipped where the reference is absent
(the GPU box).

GPU: the linked driver (the reference's own ingress and egress around
classify_on_gpu) reproduces the reference's output files byte for byte.
"""
import gzip
import os
import shutil
import subprocess

import pytest

from conftest import EDGE, GOLDEN, ROOT, edge_cases

SHIM = os.path.join(ROOT, "oracle", "_ref", "shim_driver")


@pytest.mark.skipif(not os.path.isdir("/root/reference/src"), reason="reference not present")
def test_shim_builds_against_reference_headers():
    p = subprocess.run(["make", "-B", "-s", "-f", "oracle/shim.mk"], cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    assert os.access(SHIM, os.X_OK)
    ldd = subprocess.run(["ldd", SHIM], capture_output=True, text=True).stdout
    assert "librepkiller_amd.so" in ldd


@pytest.mark.gpu
def test_shim_driver_matches_reference(tmp_path):
    if not os.path.exists(SHIM):
        pytest.skip("oracle/_ref/shim_driver not built (needs /root/reference at build time)")
    inp, out = tmp_path / "in.csv", tmp_path / "out.csv"
    with gzip.open(os.path.join(GOLDEN, "corpus10k.in.csv.gz"), "rb") as fi, \
            open(inp, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    p = subprocess.run([SHIM, str(inp), str(out), "0.3", "0.3"], capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    with gzip.open(os.path.join(GOLDEN, "corpus10k.out.csv.gz"), "rb") as f:
        assert out.read_bytes() == f.read()
    for name, case in edge_cases():
        if case["expect"] != "ref":
            continue
        p = subprocess.run([SHIM, os.path.join(EDGE, name + ".in.csv"), str(out),
                            repr(case["len_ratio"]), repr(case["pos_ratio"])],
                           capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, (name, p.stderr)
        with open(os.path.join(EDGE, name + ".out.csv"), "rb") as f:
            assert out.read_bytes() == f.read(), name
