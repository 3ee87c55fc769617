"""The kernels' Markstein division (csrc/slgpu.hip div_rn) equals IEEE division: compiled and
run on the host over random operands from the ranges the kernels use (tools/markstein_check.c).
The GPU side is covered by the bit-exact float64 XYZ parity tests (tests/test_gpu_parity.py)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_markstein_division_matches_ieee(tmp_path):
    exe = tmp_path / "markstein_check"
    subprocess.run(["gcc", "-O2", "-o", str(exe), os.path.join(ROOT, "tools", "markstein_check.c"), "-lm"],
                   check=True)
    out = subprocess.run([str(exe), "20000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches=0" in out.stdout
