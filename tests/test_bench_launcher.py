"""bench.py's own rank launcher (`--gpus N` without torchrun): the per-rank
environment, rank 0's line reaching stdout, and failure propagation.  CPU only:
the launched script here is a stand-in that never touches HIP."""
import json
import os
import subprocess
import sys
import textwrap

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_rank_env_matches_torchrun_convention():
    base = {"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    envs = [bench.rank_env(base, r, 4, 29511) for r in range(4)]
    for r, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29511"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/bin"
    assert "RANK" not in base                   # the parent's environment is untouched


def _stub(tmp_path, body):
    p = tmp_path / "stub.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def test_launcher_relays_rank0_line_and_succeeds(tmp_path):
    stub = _stub(tmp_path, """
        import json, os, sys
        if os.environ["RANK"] == "0":
            print(json.dumps({"world": int(os.environ["WORLD_SIZE"]), "argv": sys.argv[1:]}))
        else:
            print("rank output goes to stderr")
    """)
    code = f"import sys; sys.path.insert(0, {REPO!r}); import bench; sys.exit(bench.launch_ranks(['--x'], 3, {stub!r}))"
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and json.loads(lines[0]) == {"world": 3, "argv": ["--x"]}
    assert "rank output goes to stderr" in out.stderr


def test_launcher_propagates_a_failing_rank(tmp_path):
    stub = _stub(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(60)                # the others would wait at a barrier
    """)
    code = f"import sys; sys.path.insert(0, {REPO!r}); import bench; sys.exit(bench.launch_ranks([], 2, {stub!r}))"
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert out.returncode == 3


def test_parent_does_not_load_the_engine_before_spawning():
    # the launcher path returns before `pygcransac._native` is imported
    src = open(os.path.join(REPO, "bench.py")).read()
    main = src[src.index("def main():"):]
    assert main.index("launch_ranks(") < main.index("from pygcransac import _native")
