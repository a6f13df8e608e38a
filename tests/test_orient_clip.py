"""The orientation residual's range-aware angle clipping (rect.h
orient_sq_residual) is bit-identical to the general clipAngle form it
replaced (math_utils.hpp:78-102 restated): host build of the same header."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "graph-cut-ransac_amd", "csrc")


def test_range_aware_clipping_equals_general_form_bitwise(tmp_path):
    exe = str(tmp_path / "orient_clip")
    try:
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-I", CSRC,
                               os.path.join(HERE, "cpp", "orient_clip.cpp"), "-o", exe])
    except (OSError, subprocess.CalledProcessError) as e:  # pragma: no cover
        pytest.fail(f"g++ build failed: {e}")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert ", 0 mismatches" in out.stdout
