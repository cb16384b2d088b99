"""Init placement (rocmdash/runtime/placement.py): the NUMA node the process starts the
HSA runtime on is picked from per-node counter-read probes, cached per GPU and boot,
and the pin leaves the sampler threads' own NUMA-local choice intact."""

import json
import os

import pytest

from rocmdash.runtime import placement

_REAL_RUNTIME_STARTED = placement._runtime_started


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


def test_cpulist_parse():
    assert placement._cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]


def test_calibrate_picks_the_fastest_node_and_caches(monkeypatch):
    _two_nodes(monkeypatch)
    calls = []

    def probe(device, bdf, cpus, timeout_s=60.0):
        calls.append(tuple(cpus))
        return {(0, 1): 141.0, (2, 3): 71.5}[tuple(cpus)]

    monkeypatch.setattr(placement, "_probe_node", probe)
    d = placement.calibrate(0, 0x7500)
    assert d["node"] == 1 and d["source"] == "probe" and d["p50_us"] == {"0": 141.0, "1": 71.5}
    assert len(calls) == 2
    again = placement.calibrate(0, 0x7500)
    assert again["node"] == 1 and again["source"] == "cache" and len(calls) == 2
    assert placement.calibrate(0, 0x7600)["source"] == "probe"  # another GPU: its own entry


def test_failed_probes_decide_nothing_and_are_not_cached(monkeypatch):
    _two_nodes(monkeypatch)
    monkeypatch.setattr(placement, "_probe_node", lambda *a, **k: None)
    d = placement.calibrate(0, 0x7500)
    assert d["node"] is None
    assert not os.path.exists(placement._cache_path(0x7500))


def test_pin_for_init_pins_the_thread_and_remembers_the_process_mask(monkeypatch):
    _two_nodes(monkeypatch)
    monkeypatch.setattr(placement, "_probe_node", lambda d, b, cpus, timeout_s=60.0: 50.0 if cpus == [2, 3] else 90.0)
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


def test_cache_is_keyed_by_the_node_set(monkeypatch, tmp_path):
    _two_nodes(monkeypatch)
    path = placement._cache_path(0x7500)
    with open(path, "w") as f:
        json.dump({"node": 0, "p50_us": {"0": 70.0}, "source": "probe"}, f)  # written on a 1-node mask
    monkeypatch.setattr(placement, "_probe_node", lambda d, b, cpus, timeout_s=60.0: float(cpus[0]))
    assert placement.calibrate(0, 0x7500)["source"] == "probe"



def test_runtime_started_is_false_without_kfd():
    assert _REAL_RUNTIME_STARTED() is False  # a CPU test process has no /dev/kfd open


def test_probes_are_serialised_node_wide_and_the_cache_is_reread(monkeypatch):
    """8 ranks starting at once: probes never overlap (node-wide flock), and ranks of
    the same GPU that waited for the lock take the cache instead of probing again."""
    import threading
    import time

    _two_nodes(monkeypatch)
    active = []
    overlap = []
    calls = []
    lock = threading.Lock()

    def probe(device, bdf, cpus, timeout_s=60.0):
        with lock:
            active.append(1)
            if len(active) > 1:
                overlap.append(bdf)
            calls.append(bdf)
        time.sleep(0.02)
        with lock:
            active.pop()
        return 50.0 if cpus == [2, 3] else 90.0

    monkeypatch.setattr(placement, "_probe_node", probe)
    results = []

    def rank(bdf):
        results.append(placement.calibrate(0, bdf))

    # 4 GPUs x 2 ranks each (e.g. a restart racing a slow start)
    threads = [threading.Thread(target=rank, args=(0x7500 + 0x100 * (i // 2),)) for i in range(8)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not overlap, overlap
    assert len(calls) == 4 * 2  # each GPU probed once, on both nodes
    assert sorted(r["source"] for r in results) == ["cache"] * 4 + ["probe"] * 4
    assert all(r["node"] == 1 for r in results)
    assert all("lock_wait_s" in r for r in results)


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
    monkeypatch.setattr(placement, "_probe_node", lambda d, b, cpus, timeout_s=60.0: 50.0 if cpus == [2, 3] else 90.0)
    placement.pin_for_init(0, 0x7500)
    assert mask["cur"] == {2, 3}
    assert placement.restore_affinity() is True
    assert mask["cur"] == {0, 1, 2, 3}
    assert placement.restore_affinity() is False  # nothing left to undo


def test_box_wide_slow_phase_is_probed_again(monkeypatch):
    """A round where every node reads slow (a box-wide slow phase right after the box
    comes up) decides nothing: the nodes are probed again and the fast round decides
    - and only that one is cached for the boot."""
    _two_nodes(monkeypatch)
    rounds = iter([{(0, 1): 151.5, (2, 3): 149.0}, {(0, 1): 141.0, (2, 3): 72.0}])
    cur = {}

    def probe(device, bdf, cpus, timeout_s=60.0):
        if not cur or tuple(cpus) in cur["seen"]:
            cur.update(vals=next(rounds), seen=set())
        cur["seen"].add(tuple(cpus))
        return cur["vals"][tuple(cpus)]

    monkeypatch.setattr(placement, "_probe_node", probe)
    d = placement.calibrate(0, 0x7500)
    assert d["node"] == 1 and d["p50_us"] == {"0": 141.0, "1": 72.0} and not d.get("slow")
    assert d["slow_rounds"] == [{"0": 151.5, "1": 149.0}]
    assert placement.calibrate(0, 0x7500)["source"] == "cache"


def test_all_slow_calibration_is_cached_only_briefly(monkeypatch):
    _two_nodes(monkeypatch)
    calls = []
    monkeypatch.setattr(placement, "_probe_node",
                        lambda d, b, cpus, timeout_s=60.0: calls.append(1) or (150.0 if cpus == [0, 1] else 152.0))
    d = placement.calibrate(0, 0x7500)
    assert d["slow"] and d["node"] == 0 and len(calls) == 2 * placement.PROBE_ROUNDS
    assert placement.calibrate(0, 0x7500)["source"] == "cache"  # within SLOW_CACHE_S
    monkeypatch.setattr(placement, "SLOW_CACHE_S", -1.0)
    assert placement.calibrate(0, 0x7500)["source"] == "probe"  # expired: probed again
