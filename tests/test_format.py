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


def test_fast_stof_matches_strtof(tmp_path):
    """The CSV parser's fast path for the similarity column (rk::fast_stof,
    Clinger's exact m / 10^k for at most 7 significant digits) against strtof,
    which std::stof calls (FragmentsDatabase.cpp:39-40): bit-identical wherever
    it answers, over the generator's spelling, random decimals and edge forms."""
    exe = tmp_path / "stof_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "repkiller_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "stof_check.cpp"), "-o", str(exe)],
                   check=True)
    p = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "mismatches 0" in p.stdout
