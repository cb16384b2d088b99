"""Partial-node operation on the CPU (gloo): the node supervisor (rocmdash.launch ->
rocmdash.runtime.supervisor) keeps serving the GPUs that work while one fails on every
attempt, re-admits it after a backoff, and /healthz follows only the refresh loop.

Reference anchor: the reference shows whatever GPUs the exporter reports and drops a
vanished one at the next fetch (/root/reference/app.py:183-201, 262-313, 335); VERDICT r04
"what's missing" 1 / "next round" 1."""

import os

import pytest

from _supervisor_helpers import free_port, max_gap_s, outage_s, start_node, stop_node, watch

from rocmdash.runtime.supervisor import decide_culprits, restart_delay

SYNTH = ("--source", "synthetic", "--counters", "synthetic", "--refresh-hz", "10")


def test_decide_culprits():
    # a dead process is always out; with reports, the silent live members are out too
    assert decide_culprits([0, 1, 2, 3], reported=[], dead=[2]) == [2]
    assert decide_culprits([0, 1, 2, 3], reported=[0, 1, 3]) == [2]
    assert decide_culprits([0, 1, 2, 3], reported=[0, 3], dead=[1]) == [1, 2]
    # everyone reported: a transient failure, nobody excluded
    assert decide_culprits([0, 1, 2], reported=[0, 1, 2]) == []
    # no report, nobody dead: nothing to decide yet
    assert decide_culprits([0, 1], reported=[]) == []


def test_restart_backoff():
    assert [restart_delay(k, 5.0, 300.0) for k in range(0, 9)] == [0, 5, 10, 20, 40, 80, 160, 300, 300]


def test_fault_plan_always(monkeypatch):
    from rocmdash.serve import _fault_plan

    monkeypatch.setenv("ROCMDASH_FAULT", "exit:2:3")
    monkeypatch.setenv("ROCMDASH_INCARNATION", "0")
    assert _fault_plan() == ("exit", 2, 3)
    monkeypatch.setenv("ROCMDASH_INCARNATION", "1")
    assert _fault_plan() is None  # first attempt only
    monkeypatch.setenv("ROCMDASH_FAULT", "hang:2:3:always")
    assert _fault_plan() == ("hang", 2, 3)  # every attempt: a GPU that stays broken
    monkeypatch.setenv("ROCMDASH_FAULT", "startfail:1:0:always")
    assert _fault_plan() == ("startfail", 1, 0)
    monkeypatch.setenv("ROCMDASH_FAULT", "exit:2:3:sometimes")
    with pytest.raises(ValueError):
        _fault_plan()


def test_vote_flags():
    import numpy as np

    from rocmdash.serve import VOTE_REGROUP, VOTE_STOP, vote_flags

    assert vote_flags(np.array([0.0, 2.0, np.nan, 0.0])) == VOTE_REGROUP
    assert vote_flags(np.array([1.0, 2.0])) == VOTE_STOP | VOTE_REGROUP
    assert vote_flags(None) == 0


@pytest.mark.slow
@pytest.mark.parametrize("fault", ["exit", "hang"])
def test_node_keeps_serving_without_a_persistently_failing_gpu(fault, tmp_path):
    """4 ranks; GPU 2's rank dies (exit) or stops answering (hang) 30 refreshes into EVERY
    attempt. The other 3 GPUs are back on /metrics within 2 collective timeouts of the
    failure, GPU 2 shows rocmdash_gpu_up 0 with its reason, it is restarted in a fresh
    process (backoff) and re-admitted, fails again, and the node keeps serving through
    all of it with /healthz 200."""
    T = 6.0
    port = free_port()
    p = start_node(4, port, serve_args=(*SYNTH, "--collective-timeout", str(T)),
                   env={"ROCMDASH_FAULT": f"{fault}:2:30:always"}, log_path=str(tmp_path / "node.log"))
    full, partial = {"0", "1", "2", "3"}, {"0", "1", "3"}
    try:
        # the first loss and the second cycle: GPU 2 restarted at least twice
        hist, codes = watch(port, lambda h: any(s["gpus"] == full for _, s in h)
                            and h[-1][1]["restarts"].get("2", 0) >= 2 and h[-1][1]["gpus"] == partial,
                            timeout=150)
    finally:
        rc = stop_node(p)
    log = (tmp_path / "node.log").read_text()
    gap = outage_s(hist, full, partial)
    assert gap is not None and gap < 2 * T, (gap, log[-3000:])
    last = hist[-1][1]
    assert last["up"] == {"0": 1.0, "1": 1.0, "2": 0.0, "3": 1.0}, last
    assert "2" in last["down"] and ("exited" in last["down"]["2"] if fault == "exit"
                                    else "stopped answering" in last["down"]["2"]), last["down"]
    # re-admitted in between: some later refresh showed all 4 again
    first_partial = next(i for i, (_, s) in enumerate(hist) if s["gpus"] == partial)
    assert any(s["gpus"] == full for _, s in hist[first_partial:]), [sorted(s["gpus"]) for _, s in hist]
    # the node never stopped refreshing for longer than 2 collective timeouts
    assert max_gap_s(hist) < 2 * T, max_gap_s(hist)
    assert set(codes) <= {200}, codes
    assert rc == 0, log[-3000:]
    assert "excluded [2]" in log or "lost [2]" in log, log[-3000:]


@pytest.mark.slow
def test_gpu_that_never_starts_is_left_out():
    """A GPU whose rank fails while it builds its agent (HIP device refuses) on every
    attempt: the node forms without it at start-up and exports it as down."""
    port = free_port()
    p = start_node(3, port, serve_args=(*SYNTH, "--collective-timeout", "10"),
                   env={"ROCMDASH_FAULT": "startfail:1:0:always"})
    try:
        hist, codes = watch(port, lambda h: h[-1][1]["gpus"] == {"0", "2"} and h[-1][1]["restarts"].get("1", 0) >= 1,
                            timeout=120)
    finally:
        stop_node(p)
    last = hist[-1][1]
    assert last["up"]["1"] == 0.0 and "before it was ready" in last["down"]["1"], last
    assert set(codes) <= {200}, codes


@pytest.mark.slow
def test_stale_source_is_a_metric_not_a_restart():
    """A rank whose samplers stop (it keeps refreshing): rocmdash_source_stale{gpu 1} = 1
    while /healthz stays 200 (the liveness probe must not kill the node's exporter for
    one GPU's telemetry)."""
    port = free_port()
    p = start_node(2, port, serve_args=(*SYNTH, "--collective-timeout", "10"), env={"ROCMDASH_FAULT": "stall:1:3"})
    try:
        hist, codes = watch(port, lambda h: h[-1][1]["stale"].get(("1", "smi")) == 1.0, timeout=120)
        from _supervisor_helpers import get

        code, msg = get(f"http://127.0.0.1:{port}/healthz")
    finally:
        stop_node(p)
    st = hist[-1][1]["stale"]
    assert st[("1", "smi")] == 1.0 and st[("1", "counter")] == 1.0 and st[("0", "smi")] == 0.0, st
    assert code == 200 and "last refresh" in msg, (code, msg)
    assert hist[-1][1]["up"] == {"0": 1.0, "1": 1.0}


@pytest.mark.slow
def test_counter_daemon_feeds_every_rank_and_restarts():
    """``--counter-daemon on``: ONE node process publishes every GPU's counter rows (here
    synthetic) into shared-memory rings and the ranks read them (backend node-counterd)
    at the counter rate. Killing that process makes it restart; the counter rows resume
    on every rank. The node's CPU time is exported by process kind."""
    import signal
    import time

    from _supervisor_helpers import get

    from rocmdash.prom.exposition import parse_text

    port = free_port()
    p = start_node(3, port, serve_args=(*SYNTH, "--collective-timeout", "10"), env={"ROCMDASH_COUNTER_HZ": "100"},
                   counter_daemon="on")

    def samples():
        code, body = get(f"http://127.0.0.1:{port}/metrics")
        if code != 200:
            return None
        out = {"pid": None, "cpu": {}}
        for s in parse_text(body):
            d = s.label_dict()
            if s.name == "rocmdash_sampler_samples_total" and d.get("source") == "counter":
                out[d["gpu_id"]] = (s.value, d["backend"])
            elif s.name == "rocmdash_counter_daemon_pid":
                out["pid"] = int(s.value)
            elif s.name == "rocmdash_node_cpu_seconds_total":
                out["cpu"][d["process"]] = s.value
        return out

    try:
        deadline = time.monotonic() + 90
        a = None
        while time.monotonic() < deadline:
            a = samples()
            if a and all(g in a and a[g][0] > 50 for g in ("0", "1", "2")) and a["pid"]:
                break
            time.sleep(0.3)
        assert a and a["pid"], a
        assert {a[g][1] for g in ("0", "1", "2")} == {"node-counterd"}, a
        time.sleep(2.0)
        b = samples()
        rates = [(b[g][0] - a[g][0]) / 2.0 for g in ("0", "1", "2")]
        assert all(60 < r < 140 for r in rates), rates  # ~100 rows/s per GPU through the rings
        assert set(b["cpu"]) == {"supervisor", "counterd", "rank"} and b["cpu"]["rank"] > 0, b["cpu"]
        os.kill(a["pid"], signal.SIGKILL)
        deadline = time.monotonic() + 60
        c = None
        while time.monotonic() < deadline:
            c = samples()
            if c and c["pid"] and c["pid"] != a["pid"] and all(c[g][0] > b[g][0] + 50 for g in ("0", "1", "2")):
                break
            time.sleep(0.3)
        assert c and c["pid"] != a["pid"] and all(c[g][0] > b[g][0] + 50 for g in ("0", "1", "2")), (b, c)
    finally:
        stop_node(p)


@pytest.mark.slow
def test_production_measurement_reports_node_totals():
    """rocmdash.runtime.nodemeasure (bench.py's production_node): the supervised service
    measured from outside - node-total CPU by process kind, ~100 counter rows/s per GPU
    through the node counter process, and every process's PSS (the pod's memory)."""
    from rocmdash.runtime.nodemeasure import measure_production

    res = measure_production(2, seconds=3.0, counter_daemon="on", counters="synthetic", cpu=True,
                             extra_serve_args=("--source", "synthetic"), start_budget_s=120)
    assert res["error"] is None and res["rc"] == 0, res
    assert set(res["node_cpu_seconds_per_s"]) == {"supervisor", "counterd", "rank"}, res
    assert 0 < res["node_cpu_seconds_per_s_total"] < 4.0, res
    assert all(60 < r < 140 for r in res["counter_rows_per_s_by_gpu"].values()), res
    assert res["counter_backend"] == ["node-counterd"], res
    assert set(res["process_pss_mib"]) == {"supervisor", "counterd", "rank:0", "rank:1"}, res
    assert all(v > 10 for v in res["process_pss_mib"].values()), res
    # the counter process loads no torch (rocmdash.runtime.native.load(with_torch=False))
    assert res["process_pss_anon_mib"]["counterd"] < res["process_pss_anon_mib"]["rank:0"] / 2, res
    assert res["node_pss_mib"] >= sum(res["process_pss_mib"].values()) - 1, res


def test_lean_runtime_env_defaults_and_caller_wins(tmp_path):
    """The supervisor starts node processes on one hardware queue with a small scratch
    preallocation and lean RCCL buffers (profiles/r05/footprint/), unless the caller set
    those variables itself."""
    from rocmdash.runtime.supervisor import LEAN_RUNTIME_ENV, NodeSupervisor

    sup = NodeSupervisor(["true"], 1, env={"GPU_MAX_HW_QUEUES": "4", "PATH": os.environ.get("PATH", "")})
    try:
        assert sup.env["GPU_MAX_HW_QUEUES"] == "4"  # the caller's
        for k, v in LEAN_RUNTIME_ENV.items():
            if k != "GPU_MAX_HW_QUEUES":
                assert sup.env[k] == v, k
        assert LEAN_RUNTIME_ENV["HSA_SCRATCH_SINGLE_LIMIT"] == "1048576"
    finally:
        sup.shutdown(grace_s=1.0)


def test_stray_stop_vote_restarts_the_stopped_slots():
    """members that left on a stop vote while another slot was down must be
    started again (the supervisor is not stopping), or the node never re-forms; while a
    voter is still a member nothing is restarted, and with every slot stopped nothing is
    (run() exits)."""
    from rocmdash.runtime.supervisor import NodeSupervisor

    sup = NodeSupervisor(["true"], 3, env={"PATH": os.environ.get("PATH", "")})
    spawned = []
    sup._spawn = lambda s: spawned.append(s.index) or setattr(s, "state", "starting")
    try:
        sup.slots[0].state, sup.slots[1].state, sup.slots[2].state = "stopped", "member", "down"
        sup.slots[2].next_start = 1e18  # its backoff is far away
        sup.step()
        assert spawned == [] and sup.slots[0].state == "stopped"  # slot 1 has not left yet
        sup.slots[1].state = "stopped"
        sup.step()
        assert sorted(spawned) == [0, 1] and sup.slots[2].state == "down"
        spawned.clear()
        for s in sup.slots:
            s.state = "stopped"
        sup.step()
        assert spawned == []  # the node was told to stop
    finally:
        sup.shutdown(grace_s=1.0)


def test_launch_master_port_forms():
    from rocmdash.launch import store_port_from

    ign = []
    assert store_port_from(["--master-port=2345"], ign) == 2345
    assert store_port_from(["--master-port", "2346", "--nnodes=1"], ign) == 2346 and ign == ["--nnodes=1"]
    assert store_port_from(["--master_port", "2347"]) == 2347
    assert store_port_from([]) == 0
    with pytest.raises(SystemExit):
        store_port_from(["--master-port"])
    with pytest.raises(SystemExit):
        store_port_from(["--master-port", "x"])
