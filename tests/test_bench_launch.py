"""bench.py's launch contract: `--gpus N` without a
launcher runs N ranks itself (torch.distributed.run, one process per GPU,
rendezvous on 127.0.0.1) and a WORLD_SIZE that disagrees with --gpus fails
loudly.  The ranks of --launch-check join a gloo group and all-reduce on
the CPU, so the spawn path is covered without a GPU."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus_2_spawns_two_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec == {"world": 2, "rank_sum": 1.0}


def test_world_size_mismatch_fails_loudly():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=120,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_profiled_entry_guard():
    """Committed PMC / SQ entries are used only when their profiled kernel
    time can come from this build: within 15 % of the run's, plus the
    profiler's per-dispatch cost above it."""
    b = _bench_module()
    assert b.same_build_time(0.0057, 0.0046)       # C2 under the kernel trace
    assert not b.same_build_time(0.0080, 0.0046)   # another build
    assert not b.same_build_time(0.0030, 0.0046)
    assert b.same_build_time(7.63, 7.47)           # tube: the slack is negligible
    assert not b.same_build_time(9.0, 7.47)
