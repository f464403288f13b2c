"""The device q8_1 quantizer divides as fma(fma(-q, d, x), r, q) with q = x*r, r = v_rcp_f32(d)
(gguf_q8_1.hpp) instead of an IEEE division.  tools/q81_div_check.cpp proves on the host that
fp16 of that quotient equals fp16(x / d) for every pair of fp16 values a q8_1 block can hold
and every r within 1 ulp of 1/d (v_rcp_f32's accuracy bound).  CPU test: compile and run it."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_quantizer_division_exhaustive(tmp_path):
    exe = tmp_path / "q81_div_check"
    subprocess.run(["g++", "-O2", "-fopenmp", "-ffp-contract=off", "-std=c++17",
                    os.path.join(ROOT, "tools", "q81_div_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=False, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches 0" in out.stdout and "amax/127 mismatches 0" in out.stdout, out.stdout
