"""bench.py runs each rank's measurement in a child process and starts EVERY rank's
child again when any child reports that its counter reads came up in the slow driver
state (``ROCMDASH_BENCH_FAKE_SLOW=<rank>:<attempt>`` simulates it), at most --restarts
times; the last attempt measures whatever state it got. CPU / gloo here."""

import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--cpu", "--steps", "5", "--warmup", "1", "--window", "256", "--timing-steps", "0"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env)
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=e)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout
    return json.loads(lines[0]), res.stderr


def test_world1_slow_child_is_restarted():
    d, err = _run([sys.executable, "bench.py", *ARGS], ROCMDASH_BENCH_FAKE_SLOW="0:0")
    assert d["startup_restarts"] == 1 and d["slow_state"] is None, d
    assert "slow driver state" in err


def test_last_attempt_measures_whatever_it_got():
    d, _ = _run([sys.executable, "bench.py", *ARGS, "--restarts", "0"], ROCMDASH_BENCH_FAKE_SLOW="0:0")
    assert d["startup_restarts"] == 0 and d["slow_state"] and d["slow_state"]["fake"], d


def test_one_slow_rank_restarts_every_rank():
    """World 2 under torch.distributed.run: rank 1's first child is slow, so BOTH ranks
    start fresh children, which form a new group on the launcher's store."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", *ARGS]
    d, err = _run(cmd, ROCMDASH_BENCH_FAKE_SLOW="1:0")
    assert d["n_gpus"] == 2 and d["startup_restarts"] == 1, d
    assert "rank 1 attempt 0" in err


def test_no_launcher_starts_n_ranks():
    """``--gpus N`` without torch.distributed.run: the bench starts the N rank processes
    itself and the line reports N ranks, each with its own record."""
    d, err = _run([sys.executable, "bench.py", "--gpus", "4", "--cpu", "--steps", "20", "--warmup", "2", "--window",
                   "256", "--timing-steps", "0", "--e2e-s", "1"])
    assert d["n_gpus"] == 4 and len(d["ranks"]) == 4, d
    assert sorted(r["rank"] for r in d["ranks"]) == [0, 1, 2, 3]
    assert "started 4 rank processes" in err
    # interpretability fields
    assert d["cpu_seconds_per_s"] > 0 and all(r["cpu_seconds_per_s"] > 0 for r in d["ranks"])
    assert d["production_fresh_per_s_per_gpu"] > 0 and d["production_cpu_seconds_per_s"] > 0
    c = d["comparable_refresh_ms"]
    assert c["field"] == "prometheus_page_p50_ms" and c["value"] == d["prometheus_page_p50_ms"] > 0


def _rc(cmd, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env)
    return subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=120, env=e)


def test_too_few_gpus_is_an_error():
    """``--gpus 8`` where fewer GPUs are visible exits non-zero without a JSON line
    instead of measuring one GPU (here: none visible)."""
    res = _rc([sys.executable, "bench.py", "--gpus", "8", "--steps", "5"])
    assert res.returncode == 2 and "GPU(s) visible" in res.stderr, res.stderr[-2000:]
    assert not [ln for ln in res.stdout.splitlines() if ln.startswith("{")]


def test_gpus_disagreeing_with_launcher_is_an_error():
    res = _rc([sys.executable, "bench.py", "--gpus", "4", *ARGS], WORLD_SIZE="2", RANK="0")
    assert res.returncode == 2 and "WORLD_SIZE 2" in res.stderr, res.stderr[-2000:]
