"""bench.py runs each rank's measurement in a child process and starts a rank's child
again when THAT child reports that its counter reads came up in the slow driver state
(``ROCMDASH_BENCH_FAKE_SLOW=<rank>:<attempt>[,...]`` simulates it), at most --restarts
times per rank; the verdict is taken before the node's process group forms, so only the
slow ranks restart. The last attempt measures whatever state it
got. CPU / gloo here."""

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


def test_one_slow_rank_restarts_alone():
    """World 2 under torch.distributed.run: rank 1's first child is slow, so rank 1 alone
    starts a fresh child; rank 0's child waits with its agent up, then both form the
    group on the launcher's store."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", *ARGS]
    d, err = _run(cmd, ROCMDASH_BENCH_FAKE_SLOW="1:0")
    assert d["n_gpus"] == 2 and d["startup_restarts"] == 1 and d["startup_restarts_by_rank"] == [0, 1], d
    assert "rank 1 attempt 0" in err and "rank 0 attempt" not in err


def test_slow_ranks_of_eight_restart_alone():
    """8 ranks, no launcher: ranks 3 and 6 come up slow on their first attempt and rank 6
    again on its second. Exactly those children restart (3 once, 6 twice), every other
    rank keeps its first child, and ONE line reports n_gpus 8 with the per-rank attempts."""
    d, err = _run([sys.executable, "bench.py", "--gpus", "8", *ARGS, "--e2e-s", "0"],
                  ROCMDASH_BENCH_FAKE_SLOW="3:0,6:0,6:1")
    assert d["n_gpus"] == 8 and len(d["ranks"]) == 8, d
    assert d["startup_restarts_by_rank"] == [0, 0, 0, 1, 0, 0, 2, 0], d["startup_restarts_by_rank"]
    assert [r["attempt"] for r in sorted(d["ranks"], key=lambda r: r["rank"])] == [0, 0, 0, 1, 0, 0, 2, 0]
    assert d["startup_restarts"] == 3 and d["slow_state"] is None
    restarted = sorted({ln.split(":")[0] for ln in err.splitlines() if "starting attempt" in ln})
    assert restarted == ["[bench] rank 3", "[bench] rank 6"], restarted


def test_restart_plan():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert b.restart_plan([0, 1, 0, 1], [0, 0, 0, 2], budget=2) == ("restart", [1])  # rank 3 out of restarts
    assert b.restart_plan([0, 0], [0, 0], budget=2) == ("go", [])
    assert b.restart_plan([0, 1, 2], [0, 0, 0], budget=2) == ("abort", [])
    assert b.restart_plan([1, 1], [2, 2], budget=2) == ("go", [])  # slow but out of restarts: measure


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


def test_node_window_tail_and_mode_label():
    """the node-window record reports p50 / p90 / p99 of hits and
    misses apart, the miss count and where they fell, and says what ran."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    ms = [0.1] * 98 + [1.5, 2.0]
    kinds = ["hit"] * 98 + ["chain", "chain"]
    t = bench._node_window_tail(ms, kinds)
    assert t["all"]["n"] == 100 and t["all"]["p50"] == 0.1 and t["all"]["p99"] == 2.0
    assert t["hit"]["p99"] == 0.1 and t["chain"]["n"] == 2 and t["chain_refreshes"] == 2 and t["chain_at"] == [98, 99]
    assert bench._node_window_tail([], []) is None

    class N:
        long = True

    class L:
        brackets = True
        incremental = True

    assert bench._node_window_mode(N, L).startswith("node bracket mode")
    L.brackets = False
    assert bench._node_window_mode(N, L) == "distributed radix select"
    N.long = False
    assert bench._node_window_mode(N, None) == "sorted windows all-gathered + rank selection"
