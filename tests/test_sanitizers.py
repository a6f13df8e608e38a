"""Sanitizer builds of the engine's host-side concurrency (CPU suite).

Round 5 saw two host memory-safety faults in the product (DESIGN §11,
item 1): a heap overflow from the final refit's rectified-angle lambda
writing into the pool workers' own thread_local vectors (csrc/host_fit.cpp,
fixed in 9a868b3), and two jobs running at once in the host pool after a
begin()/end() lock race (fixed in 73ef833).  These tests build the pool
(csrc/host_pool.h, header-only, no HIP) and the host fits / graph-cut jobs
that run on it under ThreadSanitizer and AddressSanitizer + UBSan:

* ``tests/cpp/host_pool.cpp``: concurrent callers hammering parallel_for,
  begin/end with nested calls, nested jobs and throwing jobs;
* ``tests/cpp/fit_pool.cpp``: LO-sized fits on the workers, then big refits
  whose angles go through the pool, bitwise against the serial fit;
* ``tests/cpp/gc_jobs.cpp`` / ``gc_clique.cpp``: the graph-cut labeling jobs
  (4 threads) and the clique closed form.

Two canaries show the harness catches both round-5 faults: the pre-fix pool
(``tests/cpp/host_pool_prefix.h``) must be reported by TSan, and the pre-fix
angle lambda (host_fit.cpp with the thread_local named inside the lambda,
patched into a temporary copy) must be reported by ASan.
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "graph-cut-ransac_amd", "csrc")
INC = os.path.join(ROOT, "include")
CPP = os.path.join(HERE, "cpp")

BASE = ["g++", "-std=c++17", "-O1", "-g", "-ffp-contract=off", "-fno-fast-math", "-pthread",
        "-fno-omit-frame-pointer", "-I", CSRC, "-I", INC]
SAN = {
    "thread": ["-fsanitize=thread"],
    "address": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"],
}
ENV = {
    "thread": {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"},
    "address": {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "UBSAN_OPTIONS": "print_stacktrace=1"},
}

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


def _build(tmp_path, san, name, sources, extra=()):
    exe = str(tmp_path / f"{name}_{san}")
    cmd = BASE + SAN[san] + list(extra) + list(sources) + ["-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, "build failed:\n" + r.stderr[-4000:]
    return exe


def _run(exe, san, args=(), timeout=240):
    env = dict(os.environ)
    env.update(ENV[san])
    return subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.parametrize("san", ["thread", "address"])
def test_host_pool_hammer(tmp_path, san):
    exe = _build(tmp_path, san, "host_pool", [os.path.join(CPP, "host_pool.cpp")])
    r = _run(exe, san, (8, 3000, 8))
    assert r.returncode == 0, r.stdout + r.stderr[-6000:]
    assert r.stdout.startswith("OK"), r.stdout


def test_prefix_pool_is_reported_by_tsan(tmp_path):
    # the round-5 begin()/end() (shared unique_lock member): TSan must see it
    exe = _build(tmp_path, "thread", "host_pool_prefix", [os.path.join(CPP, "host_pool.cpp")],
                 extra=["-DGCR_PREFIX_POOL"])
    try:
        r = _run(exe, "thread", (8, 3000, 8), timeout=60)
        out = r.stdout + r.stderr
        caught = r.returncode != 0 and ("ThreadSanitizer" in out or "FAIL" in out)
    except subprocess.TimeoutExpired:
        caught = True                 # pending_ underflow: the old pool hangs in its wait
    assert caught, "the pre-fix pool ran clean under TSan: the hammer no longer exercises the race"


@pytest.mark.parametrize("san", ["thread", "address"])
def test_host_fits_on_the_pool(tmp_path, san):
    exe = _build(tmp_path, san, "fit_pool",
                 [os.path.join(CPP, "fit_pool.cpp"), os.path.join(CSRC, "host_fit.cpp")])
    r = _run(exe, san)
    assert r.returncode == 0, r.stdout + r.stderr[-6000:]
    assert r.stdout.startswith("OK"), r.stdout


def test_prefix_refit_angles_are_reported_by_asan(tmp_path):
    # host_fit.cpp with the round-5 bug put back: the thread_local angle
    # scratch named inside the lambda the pool runs
    src = open(os.path.join(CSRC, "host_fit.cpp")).read()
    fixed = ("    thread_local std::vector<double> tl_ang, tl_wts;\n"
             "    std::vector<double>& ang = tl_ang;\n"
             "    std::vector<double>& wts = tl_wts;\n")
    assert fixed in src, "fit_sift22's angle scratch changed: update this canary"
    bad = tmp_path / "host_fit_prefix.cpp"
    bad.write_text(src.replace(fixed, "    thread_local std::vector<double> ang, wts;\n"))
    exe = _build(tmp_path, "address", "fit_pool_prefix", [os.path.join(CPP, "fit_pool.cpp"), str(bad)])
    r = _run(exe, "address")
    assert r.returncode != 0 and "AddressSanitizer" in r.stderr, r.stdout + r.stderr[-3000:]


@pytest.mark.parametrize("san", ["thread", "address"])
def test_graphcut_jobs(tmp_path, san):
    exe = _build(tmp_path, san, "gc_jobs", [os.path.join(CPP, "gc_jobs.cpp")])
    r = _run(exe, san, (8,))
    assert r.returncode == 0, r.stdout + r.stderr[-6000:]
    assert "mismatches 0" in r.stdout


def test_graphcut_clique_asan(tmp_path):
    exe = _build(tmp_path, "address", "gc_clique", [os.path.join(CPP, "gc_clique.cpp")])
    r = _run(exe, "address", (200000,))
    assert r.returncode == 0, r.stdout + r.stderr[-6000:]
    assert "mismatches 0" in r.stdout
