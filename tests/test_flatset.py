"""The host-side id set and id -> slot map of the AMR bookkeeping
(dccrg_amd/csrc/flatset.hpp) against std::set / std::map: random inserts,
erases and lookups (CPU)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_flatset_matches_std_set(tmp_path):
    exe = str(tmp_path / "flatset_test")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(ROOT, "dccrg_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "flatset_test.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "PASS" in out.stdout, out.stdout + out.stderr
