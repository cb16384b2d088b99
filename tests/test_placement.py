"""Init placement (rocmdash/runtime/placement.py): the NUMA node the process starts the
HSA runtime on is picked from counter-read probes - one probe child per NUMA node for
the WHOLE node, every GPU timed, cached by bdf per boot - and the pin leaves the sampler
threads' own NUMA-local choice intact."""

import json
import os
import re
import threading
import time

import pytest

from rocmdash.runtime import placement

_REAL_RUNTIME_STARTED = placement._runtime_started
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GPUS = ["7500", "7600", "7700", "7800", "7900", "7a00", "7b00", "7c00"]


@pytest.fixture(autouse=True)
def _fresh(monkeypatch, tmp_path):
    monkeypatch.setattr(placement, "_original_mask", None)
    monkeypatch.setattr(placement, "_choice", None)
    monkeypatch.setattr(placement.tempfile, "gettempdir", lambda: str(tmp_path))
    monkeypatch.delenv("ROCMDASH_INIT_PLACEMENT", raising=False)
    monkeypatch.setattr(placement, "_runtime_started", lambda: False)
    monkeypatch.setattr(placement, "RETRY_PAUSE_S", 0.0)
    yield


def _two_nodes(monkeypatch):
    nodes = {0: [0, 1], 1: [2, 3]}
    monkeypatch.setattr(placement, "numa_nodes", lambda: dict(nodes))
    return nodes


def _node_probe(table, calls=None):
    """A fake probe child: {cpus: {bdf: us}} -> _probe_node(cpus)."""

    def probe(cpus, timeout_s=60.0):
        if calls is not None:
            calls.append(tuple(cpus))
        return dict(table[tuple(cpus)])

    return probe


def test_cpulist_parse():
    assert placement._cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]


def test_one_calibration_serves_every_gpu_of_the_node(monkeypatch):
    _two_nodes(monkeypatch)
    calls = []
    monkeypatch.setattr(placement, "_probe_node", _node_probe(
        {(0, 1): {"7500": 141.0, "7600": 70.0}, (2, 3): {"7500": 71.5, "7600": 139.0}}, calls))
    d = placement.calibrate(0, 0x7500)
    assert d["node"] == 1 and d["source"] == "probe" and d["p50_us"] == {"0": 141.0, "1": 71.5}
    assert d["gpus_calibrated"] == 2 and len(calls) == 2
    again = placement.calibrate(0, 0x7500)
    assert again["node"] == 1 and again["source"] == "cache" and len(calls) == 2
    other = placement.calibrate(1, 0x7600)  # another GPU: same calibration, its own best node
    assert other["source"] == "cache" and other["node"] == 0 and len(calls) == 2


def test_failed_probes_decide_nothing_and_are_not_cached(monkeypatch):
    _two_nodes(monkeypatch)
    monkeypatch.setattr(placement, "_probe_node", lambda *a, **k: None)
    d = placement.calibrate(0, 0x7500)
    assert d["node"] is None
    assert not os.path.exists(placement._cache_path())


def test_pin_for_init_pins_the_thread_and_remembers_the_process_mask(monkeypatch):
    _two_nodes(monkeypatch)
    monkeypatch.setattr(placement, "_probe_node", _node_probe({(0, 1): {"7500": 90.0}, (2, 3): {"7500": 50.0}}))
    pinned = []
    monkeypatch.setattr(placement.os, "sched_getaffinity", lambda pid: {0, 1, 2, 3})
    monkeypatch.setattr(placement.os, "sched_setaffinity", lambda pid, cpus: pinned.append(list(cpus)))
    d = placement.pin_for_init(0, 0x7500)
    assert d["node"] == 1 and pinned == [[2, 3]]
    assert placement.process_cpus() == {0, 1, 2, 3}  # what the sampler threads pick from
    assert placement.choice() is d


def test_pin_for_init_off_forced_and_without_gpu(monkeypatch):
    _two_nodes(monkeypatch)
    pinned = []
    monkeypatch.setattr(placement.os, "sched_getaffinity", lambda pid: {0, 1, 2, 3})
    monkeypatch.setattr(placement.os, "sched_setaffinity", lambda pid, cpus: pinned.append(list(cpus)))
    monkeypatch.setattr(placement, "_probe_node", lambda *a, **k: pytest.fail("no probe expected"))
    assert placement.pin_for_init(0, 0) is None  # no GPU (CPU container): nothing happens
    monkeypatch.setenv("ROCMDASH_INIT_PLACEMENT", "0")
    assert placement.pin_for_init(0, 0x7500) is None and pinned == []
    monkeypatch.setenv("ROCMDASH_INIT_PLACEMENT", "1")
    d = placement.pin_for_init(0, 0x7500)
    assert d["source"] == "ROCMDASH_INIT_PLACEMENT" and pinned == [[2, 3]]


def test_cache_is_keyed_by_the_node_set(monkeypatch):
    _two_nodes(monkeypatch)
    with open(placement._cache_path(), "w") as f:  # written on a 1-node mask
        json.dump({"nodes": [0], "gpus": {"7500": {"node": 0, "p50_us": {"0": 70.0}}}}, f)
    monkeypatch.setattr(placement, "_probe_node", _node_probe({(0, 1): {"7500": 90.0}, (2, 3): {"7500": 50.0}}))
    assert placement.calibrate(0, 0x7500)["source"] == "probe"


def test_runtime_started_is_false_without_kfd():
    assert _REAL_RUNTIME_STARTED() is False  # a CPU test process has no /dev/kfd open


def _startup_budget_s() -> float:
    """The exporter DaemonSet's startupProbe budget: failureThreshold x periodSeconds."""
    with open(os.path.join(ROOT, "deploy", "k8s", "exporter-daemonset.yaml")) as f:
        text = f.read()
    block = text[text.index("startupProbe:"):]
    block = block[: block.index("livenessProbe:")] if "livenessProbe:" in block else block
    period = float(re.search(r"periodSeconds:\s*(\d+)", block).group(1))
    fails = float(re.search(r"failureThreshold:\s*(\d+)", block).group(1))
    return period * fails


def test_eight_ranks_share_one_probe_set_within_the_startup_budget(monkeypatch):
    """A full node starting: 8 ranks (one per GPU) calibrate at once. The probes never
    overlap (node-wide flock), exactly ONE probe child runs per NUMA node, the 7 ranks
    that waited take the cache - and even the worst case (every round slow: 3 rounds)
    stays far inside the DaemonSet's startupProbe budget. Probe children are modelled
    at CHILD_S = 6 s (measured: 2.35 s per child timing one GPU on an MI355X box,
    profiles/r03/pass1/placement_probe_all.json; 8 GPUs add 8 x 230 reads and 7 more
    counting contexts), slept at 1/SCALE of that to keep the test fast."""
    CHILD_S, SCALE = 6.0, 100.0
    _two_nodes(monkeypatch)
    active, overlap, calls = [], [], []
    lock = threading.Lock()
    slow_rounds = {"left": 0}

    def probe(cpus, timeout_s=60.0):
        with lock:
            active.append(1)
            if len(active) > 1:
                overlap.append(tuple(cpus))
            calls.append(tuple(cpus))
        time.sleep(CHILD_S / SCALE)
        with lock:
            active.pop()
            slow = slow_rounds["left"] > 0
            if slow and tuple(cpus) == (2, 3):
                slow_rounds["left"] -= 1
        base = 150.0 if slow else 0.0
        return {b: base + (50.0 if cpus == [2, 3] else 90.0) + i for i, b in enumerate(GPUS)}

    monkeypatch.setattr(placement, "_probe_node", probe)
    budget = _startup_budget_s()
    for worst in (False, True):
        calls.clear()
        if os.path.exists(placement._cache_path()):
            os.remove(placement._cache_path())
        slow_rounds["left"] = placement.PROBE_ROUNDS if worst else 0
        results = []
        t0 = time.perf_counter()
        threads = [threading.Thread(target=lambda b=b: results.append(placement.calibrate(0, int(b, 16))))
                   for b in GPUS]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        real = time.perf_counter() - t0
        # the probe children's time at the modelled CHILD_S; everything else (lock polls,
        # cache reads, thread start-up) as it really took
        wall = len(calls) * CHILD_S + max(0.0, real - len(calls) * CHILD_S / SCALE)
        assert not overlap, overlap
        rounds = placement.PROBE_ROUNDS if worst else 1
        assert len(calls) == 2 * rounds  # one child per NUMA node per round, for all 8 GPUs
        assert sorted(r["source"] for r in results) == ["cache"] * 7 + ["probe"]
        assert all(r["node"] == 1 for r in results)
        assert wall < 0.5 * budget, (wall, budget)  # half the budget left for HIP, RCCL, 1st refresh
    assert budget >= 2 * placement.PROBE_ROUNDS * CHILD_S


def test_node_lock_times_out_instead_of_blocking(tmp_path):
    path = str(tmp_path / "x.lock")
    with placement.node_lock(path=path) as held:
        assert held
        with placement.node_lock(timeout_s=0.2, path=path) as held2:
            assert held2 is False


def test_restore_affinity_undoes_the_init_pin(monkeypatch):
    _two_nodes(monkeypatch)
    mask = {"cur": {0, 1, 2, 3}}
    monkeypatch.setattr(placement.os, "sched_getaffinity", lambda pid: set(mask["cur"]))
    monkeypatch.setattr(placement.os, "sched_setaffinity", lambda pid, cpus: mask.__setitem__("cur", set(cpus)))
    monkeypatch.setattr(placement, "_probe_node", _node_probe({(0, 1): {"7500": 90.0}, (2, 3): {"7500": 50.0}}))
    placement.pin_for_init(0, 0x7500)
    assert mask["cur"] == {2, 3}
    assert placement.restore_affinity() is True
    assert mask["cur"] == {0, 1, 2, 3}
    assert placement.restore_affinity() is False  # nothing left to undo


def test_box_wide_slow_phase_is_probed_again(monkeypatch):
    """A round where every node reads slow for some GPU (a box-wide slow phase right
    after the box comes up) decides nothing: the node is probed again and the fast round
    decides - and only that one is cached for the boot."""
    _two_nodes(monkeypatch)
    rounds = iter([{(0, 1): {"7500": 151.5}, (2, 3): {"7500": 149.0}},
                   {(0, 1): {"7500": 141.0}, (2, 3): {"7500": 72.0}}])
    cur = {}

    def probe(cpus, timeout_s=60.0):
        if not cur or tuple(cpus) in cur["seen"]:
            cur.update(vals=next(rounds), seen=set())
        cur["seen"].add(tuple(cpus))
        return dict(cur["vals"][tuple(cpus)])

    monkeypatch.setattr(placement, "_probe_node", probe)
    d = placement.calibrate(0, 0x7500)
    assert d["node"] == 1 and d["p50_us"] == {"0": 141.0, "1": 72.0} and not d.get("slow")
    assert d["slow_rounds"] == [{"0": {"7500": 151.5}, "1": {"7500": 149.0}}]
    assert placement.calibrate(0, 0x7500)["source"] == "cache"


def test_all_slow_calibration_is_cached_only_briefly(monkeypatch):
    """Rounds that neither separate the nodes nor agree with one another (a transient
    phase): no decision, cached only for SLOW_CACHE_S."""
    _two_nodes(monkeypatch)
    calls = []
    vals = iter([150.0, 152.0, 110.0, 108.0, 190.0, 185.0] * 3)
    monkeypatch.setattr(placement, "_probe_node", lambda cpus, timeout_s=60.0: calls.append(1) or {"7500": next(vals)})
    d = placement.calibrate(0, 0x7500)
    assert d["slow"] and len(calls) == 2 * placement.PROBE_ROUNDS
    assert placement.calibrate(0, 0x7500)["source"] == "cache"  # within SLOW_CACHE_S
    monkeypatch.setattr(placement, "SLOW_CACHE_S", -1.0)
    assert placement.calibrate(0, 0x7500)["source"] == "probe"  # expired: probed again


def test_uniform_box_is_a_decision_not_a_slow_phase(monkeypatch):
    """Every round reads the nodes alike AND the rounds agree: the box has no NUMA
    effect - cached for the boot like any decision (no re-probe on every start)."""
    _two_nodes(monkeypatch)
    monkeypatch.setattr(placement, "_probe_node",
                        lambda cpus, timeout_s=60.0: {"7500": 80.0 if cpus == [0, 1] else 82.0})
    d = placement.calibrate(0, 0x7500)
    assert not d.get("slow") and d["node"] == 0
    with open(placement._cache_path()) as f:
        doc = json.load(f)
    assert doc["gpus"]["7500"].get("uniform") and not doc.get("slow")
    monkeypatch.setattr(placement, "SLOW_CACHE_S", -1.0)
    assert placement.calibrate(0, 0x7500)["source"] == "cache"


@pytest.mark.parametrize("fast,slow", [(81.3, 149.7), (105.6, 200.9), (80.3, 151.0)])
def test_calibration_is_relative_to_the_counter_set(monkeypatch, fast, slow):
    """The decision does not depend on what a read costs, only on the NUMA ratio: the
    round-4 6-counter set (81 / 150 us), round 5's 7-counter set (106 / 201 us,
    profiles/r06/counter_ab/) and round 6's set all decide in ONE round, not slow
    (the 7-counter set made every calibration 'slow' - 3 rounds,
    15 s, a 60 s cache); the bench's slow-start reference is the calibrated read."""
    _two_nodes(monkeypatch)
    calls = []
    monkeypatch.setattr(placement, "_probe_node", _node_probe({(0, 1): {"7500": slow}, (2, 3): {"7500": fast}}, calls))
    d = placement.calibrate(0, 0x7500)
    assert d["node"] == 1 and not d.get("slow") and "slow_rounds" not in d and len(calls) == 2
    assert placement.fast_reference_us(d) == fast
    assert placement.fast_reference_us({"node": None}) is None


def test_probe_merges_into_the_node_cache(monkeypatch):
    """A probe that sees fewer GPUs (one the child could not open) keeps the cached
    entries of the others instead of erasing them."""
    _two_nodes(monkeypatch)
    monkeypatch.setattr(placement, "_probe_node", _node_probe(
        {(0, 1): {"7500": 141.0, "7600": 70.0}, (2, 3): {"7500": 71.5, "7600": 139.0}}))
    placement.calibrate(0, 0x7500)
    monkeypatch.setattr(placement, "_probe_node", _node_probe({(0, 1): {"7700": 72.0}, (2, 3): {"7700": 140.0}}))
    d = placement.calibrate(2, 0x7700, use_cache=False)
    assert d["node"] == 0
    with open(placement._cache_path()) as f:
        gpus = json.load(f)["gpus"]
    assert set(gpus) == {"7500", "7600", "7700"} and gpus["7500"]["node"] == 1


def test_probe_child_sees_every_gpu(monkeypatch):
    """The probe child drops per-rank device visibility: it calibrates the node."""
    seen = {}

    class Res:
        stdout = '{"p50_us": {"7500": 70.0}}\n'

    def fake_run(cmd, capture_output, text, timeout, env):
        seen.update(env)
        return Res()

    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "3")
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "3")
    monkeypatch.setattr(placement.subprocess, "run", fake_run)
    assert placement._probe_node([0, 1]) == {"7500": 70.0}
    assert "HIP_VISIBLE_DEVICES" not in seen and "ROCR_VISIBLE_DEVICES" not in seen
