"""k_score_fm's packed-fp32 rectification pre-band (csrc/kernels.hip
RPairBand) never rejects a pair the fp64 band keeps: tests/cpp/band_f32.cpp
restates both per lane on the host (fmaf correctly rounded, no contraction)
and checks random pairs plus pairs placed on the fp64 band's edges (to the
last ulp for scale, by bisection for orientation), t near 0, scale-range
limits, huge / NaN coordinates, subnormal model terms and extreme alpha.
The GPU side of the same claim is the bitwise parity of every rectification
test (the survivors only feed the exact pass)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_fp32_pre_band_is_conservative(tmp_path):
    exe = str(tmp_path / "band_f32")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                           os.path.join(HERE, "cpp", "band_f32.cpp"), "-o", exe])
    out = subprocess.run([exe, "400"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "violations 0" in out.stdout
    # the pre-band still does its job on the drawn pairs
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("drawn pairs only")][0]
    nums = [int(t.strip(",;")) for t in line.replace(",", " ").split() if t.strip(",;").isdigit()]
    r64s, r32s, r64o, r32o = nums
    assert r32s > 0.7 * r64s and r32o > 0.8 * r64o, line
