"""Shared fixtures.  `-m gpu` tests need a gfx950 device; everything else runs on CPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
EDGE = os.path.join(GOLDEN, "edge")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU")
    config.addinivalue_line("markers", "slow: larger parity sizes")


@pytest.fixture(scope="session", autouse=True)
def built():
    """Build the product library and the oracle restatement once per session."""
    lib = os.path.join(ROOT, "repkiller_amd", "librepkiller_amd.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "repkiller_amd", "csrc"), "-j8"],
                       check=True)
    if not os.path.exists(os.path.join(ROOT, "oracle", "_build", "librk_oracle.so")):
        subprocess.run(["make", "-s", "-f", "oracle/oracle.mk"], cwd=ROOT, check=True)


def edge_cases():
    with open(os.path.join(EDGE, "manifest.json")) as f:
        man = json.load(f)
    return sorted(man.items())


@pytest.fixture(scope="session")
def gpu_ctx():
    import repkiller_amd as rk
    ctx = rk.Context(0)
    yield ctx
    ctx.close()


@pytest.fixture(scope="session")
def generic_ctx():
    import repkiller_amd as rk
    ctx = rk.Context(0)
    ctx.set_pipeline("generic")
    yield ctx
    ctx.close()


@pytest.fixture(params=["record", "generic"])
def pctx(request, gpu_ctx, generic_ctx):
    """Both device pipelines (the record pipeline where inputs pack into 16-B
    records -- gpu_ctx's default -- and the generic one)."""
    return gpu_ctx if request.param == "record" else generic_ctx
