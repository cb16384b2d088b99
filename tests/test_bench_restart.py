"""bench.py at N = 1 runs the measurement in a child process and starts a fresh one
when the child reports the slow driver state (exit 75), at most --restarts times."""

import importlib.util
import os
import subprocess
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_restarts_until_a_child_is_not_slow(monkeypatch):
    bench = _bench()
    calls = []

    def fake_run(cmd, env=None, **kw):
        calls.append((env["ROCMDASH_BENCH_ATTEMPT"], env["ROCMDASH_BENCH_LAST"]))
        return types.SimpleNamespace(returncode=bench.EXIT_SLOW_STATE if len(calls) < 3 else 0)

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.delenv("ROCMDASH_BENCH_CHILD", raising=False)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.main(["--steps", "5"]) == 0
    assert calls == [("0", "0"), ("1", "0"), ("2", "1")]  # the last attempt must measure whatever it gets


def test_no_restart_loop_under_torchrun_or_cpu(monkeypatch):
    bench = _bench()
    monkeypatch.setattr(subprocess, "run", lambda *a, **k: (_ for _ in ()).throw(AssertionError("spawned")))
    monkeypatch.setenv("WORLD_SIZE", "2")
    called = {}
    monkeypatch.setattr(bench, "_run_with_restarts", lambda argv: called.setdefault("x", 1))
    # WORLD_SIZE 2 goes straight to the measurement (here: argument parsing fails fast)
    try:
        bench.main(["--definitely-not-a-flag"])
    except SystemExit:
        pass
    assert "x" not in called
    monkeypatch.setenv("WORLD_SIZE", "1")
    try:
        bench.main(["--cpu", "--definitely-not-a-flag"])
    except SystemExit:
        pass
    assert "x" not in called
