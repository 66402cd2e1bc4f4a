"""The egress float formatter (rk_format.h) against snprintf("%.6g"), which is
what ostream << float prints (commonFunctions.cpp:103)."""
import os
import subprocess

from conftest import ROOT


def test_fast_float_format_matches_printf(tmp_path):
    exe = tmp_path / "format_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "repkiller_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "format_check.cpp"), "-o", str(exe)],
                   check=True)
    p = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "mismatches 0" in p.stdout
