"""Per-GPU failure isolation of the node counter process: one lane
(native thread) per GPU in ``ShmPublisher``, the supervisor's heartbeat watch
(rocmdash.runtime.lanes.LaneWatch) and fresh lanes after a backoff.

Reference anchor: a GPU's series stand alone in the reference - each result row is parsed
on its own and a missing GPU drops out (/root/reference/app.py:183-201, 335)."""

import os
import time

import pytest

from rocmdash.runtime.lanes import LaneWatch, read_control, read_ring_header, write_control

SYNTH = ("--source", "synthetic", "--counters", "synthetic", "--refresh-hz", "10")


def _hdr(beat_s, lane=0, pid=100):
    return {"pid": pid, "lane": lane, "head": 1, "beat_ns": int(beat_s * 1e9) if beat_s is not None else 0,
            "failures": 0}


def test_lane_watch_marks_only_the_stalled_gpu_and_backs_off():
    w = LaneWatch([0, 1, 2], hz=100.0, base_s=1.0, max_s=8.0)
    assert w.stall_s == 0.25
    wall = 1000.0
    # all fresh
    assert w.update(0.0, {d: _hdr(wall - 0.01) for d in (0, 1, 2)}, wall_ns=int(wall * 1e9)) is None
    assert w.down() == {}
    # device 1 stops beating; the others go on
    t = 0.5
    hdr = {0: _hdr(wall + t - 0.01), 1: _hdr(wall), 2: _hdr(wall + t - 0.005)}
    assert w.update(t, hdr, wall_ns=int((wall + t) * 1e9)) is None
    assert set(w.down()) == {1} and "stalled" in w.down()[1]
    # before the backoff: nothing asked
    assert w.update(1.0, hdr, wall_ns=int((wall + 1.0) * 1e9)) is None
    # backoff (1 s) over: a fresh lane 1 is asked for
    ask = w.update(1.6, hdr, wall_ns=int((wall + 1.6) * 1e9))
    assert ask == {1: 1}
    # the fresh lane stalls too (never beats): failure 2, backoff 2 s
    hdr[1] = _hdr(None, lane=1)

    def at(t):
        hdr[0], hdr[2] = _hdr(wall + t - 0.01), _hdr(wall + t - 0.002)
        return w.update(t, hdr, wall_ns=int((wall + t) * 1e9))

    assert at(1.7) is None
    assert at(2.0) is None
    assert w.lanes[1].failures == 2 and "again" in w.lanes[1].reason
    assert at(3.0) is None  # backoff 2 s not over
    assert at(4.1) == {1: 2}
    # lane 2 beats: device 1 is up again
    hdr[1] = _hdr(wall + 4.2, lane=2)
    assert at(4.25) is None
    assert w.down() == {} and w.lanes[1].stalls == 2 and w.lanes[1].readmissions == 2


def test_lane_watch_whole_process_stall_is_not_per_gpu():
    w = LaneWatch([0, 1], hz=100.0)
    wall = 50.0
    hdr = {0: _hdr(wall), 1: _hdr(wall)}
    w.update(0.0, hdr, wall_ns=int(wall * 1e9))
    # both stop: no per-GPU decision (no lane is fresh), but the process counts as wedged
    assert w.update(20.0, hdr, wall_ns=int((wall + 20) * 1e9)) is None
    assert w.down() == {}
    assert w.whole_process_stalled(20.0, hdr, 10.0, wall_ns=int((wall + 20) * 1e9))
    assert not w.whole_process_stalled(20.0, hdr, 30.0, wall_ns=int((wall + 20) * 1e9))


def test_lane_watch_new_process_resets_requests():
    w = LaneWatch([0, 1], hz=100.0, base_s=0.1)
    wall = 10.0
    w.update(0.0, {0: _hdr(wall), 1: _hdr(wall)}, wall_ns=int(wall * 1e9))
    w.update(1.0, {0: _hdr(wall + 1.0), 1: _hdr(wall)}, wall_ns=int((wall + 1.0) * 1e9))
    assert w.update(1.2, {0: _hdr(wall + 1.2), 1: _hdr(wall)}, wall_ns=int((wall + 1.2) * 1e9)) == {1: 1}
    # the counter process restarts (new pid, lanes at generation 0): requests are dropped
    ask = w.update(2.0, {0: _hdr(wall + 2.0, pid=200), 1: _hdr(wall + 2.0, pid=200)}, wall_ns=int((wall + 2.0) * 1e9))
    assert ask == {} and w.down() == {}


def test_lane_watch_waits_while_rings_change_hands():
    """A restarted counter process renames its rings over the dead one's one by one: while
    the pids differ nothing is judged (the dead process's old beats are no stall)."""
    w = LaneWatch([0, 1], hz=100.0, base_s=0.1)
    wall = 10.0
    w.update(0.0, {0: _hdr(wall), 1: _hdr(wall)}, wall_ns=int(wall * 1e9))
    # the old process died 5 s ago; the new one's ring 0 beats, ring 1 is still the old file
    assert w.update(5.0, {0: _hdr(wall + 5.0, pid=300), 1: _hdr(wall)}, wall_ns=int((wall + 5.0) * 1e9)) is None
    assert w.down() == {}
    assert w.update(5.1, {0: _hdr(wall + 5.1, pid=300), 1: _hdr(wall + 5.09, pid=300)},
                    wall_ns=int((wall + 5.1) * 1e9)) is None
    assert w.down() == {}


def test_control_file_round_trip(tmp_path):
    assert read_control(str(tmp_path)) == {}
    write_control(str(tmp_path), {1: 3, 4: 1})
    assert read_control(str(tmp_path)) == {1: 3, 4: 1}


def test_publisher_lanes_are_independent_and_replaceable(tmp_path):
    """Native: a hanging source stops only its own lane; replace() gives that GPU a new
    ring (new inode, lane generation 1) whose rows flow again; the header words the
    supervisor reads from Python match the native ring."""
    from rocmdash.runtime import native

    nat = native.load(with_torch=False)
    paths = [str(tmp_path / f"r{d}.ring") for d in range(3)]
    srcs = [nat.make_synthetic_source("counter", 11 + d) for d in range(3)]
    srcs[1] = nat.make_hanging_source(srcs[1], 0.2)
    pub = nat.ShmPublisher(paths, srcs, 200.0)
    pub.start()
    try:
        time.sleep(0.8)
        h = [read_ring_header(p) for p in paths]
        assert all(x is not None and x["pid"] == os.getpid() for x in h), h
        st = pub.stats()
        # lanes 0 and 2 ran the whole time at ~200 Hz; lane 1 stopped after ~0.2 s
        assert st[0][0] > 100 and st[2][0] > 100, st
        assert st[1][0] < 70 and st[1][6] > 0.3, st  # in a read for > 0.3 s
        assert h[1]["beat_ns"] and (time.time_ns() - h[1]["beat_ns"]) * 1e-9 > 0.3
        assert (time.time_ns() - h[0]["beat_ns"]) * 1e-9 < 0.1
        assert h[0]["head"] == int(st[0][0]) or abs(h[0]["head"] - st[0][0]) <= 2
        ino = os.stat(paths[1]).st_ino
        gen = pub.replace(1, nat.make_synthetic_source("counter", 99))
        assert gen == 1
        time.sleep(0.4)
        h1 = read_ring_header(paths[1])
        assert os.stat(paths[1]).st_ino != ino and h1["lane"] == 1 and h1["head"] > 40, h1
        assert pub.stats()[1][5] == 1.0
    finally:
        t0 = time.monotonic()
        pub.stop(0.5)  # lane 1's first generation is still blocked: left behind, not joined
        assert time.monotonic() - t0 < 2.0


def test_counterd_hang_plan(monkeypatch):
    from rocmdash.runtime.counterd import hang_plan
    from rocmdash.serve import _fault_plan

    monkeypatch.setenv("ROCMDASH_FAULT", "ctrhang:1:3")
    assert hang_plan([0, 1, 2]) == {1: (3.0, False)}
    assert hang_plan([0, 2]) == {}
    assert _fault_plan() is None  # the ranks ignore the counter process's fault
    monkeypatch.setenv("ROCMDASH_FAULT", "ctrhang:2:0.5:always")
    assert hang_plan([2]) == {2: (0.5, True)}
    monkeypatch.setenv("ROCMDASH_FAULT", "exit:1:3")
    assert hang_plan([1]) == {}
    monkeypatch.setenv("ROCMDASH_FAULT", "ctrhang:1")
    with pytest.raises(ValueError):
        hang_plan([1])


@pytest.mark.slow
def test_one_hung_counter_read_keeps_the_other_gpus_flowing(tmp_path):
    """3 synthetic GPUs; device 1's counter reads block 4 s into the counter process's
    life (``ROCMDASH_FAULT=ctrhang:1:4``, first lane only). GPUs 0 and 2 keep ~100
    counter rows/s on /metrics throughout; GPU 1 is exported as
    rocmdash_counter_source_up 0 with the reason within 1 s of its last row and its
    counter series are flagged stale; /healthz stays 200; after the backoff GPU 1 gets a
    fresh lane and its rows flow again."""
    from _supervisor_helpers import free_port, get, start_node, stop_node

    from rocmdash.prom.exposition import parse_text

    port = free_port()
    p = start_node(3, port, serve_args=(*SYNTH, "--collective-timeout", "10"),
                   env={"ROCMDASH_COUNTER_HZ": "100", "ROCMDASH_FAULT": "ctrhang:1:4"}, counter_daemon="on",
                   restart_base_s=3.0, log_path=str(tmp_path / "node.log"))

    def scrape():
        code, body = get(f"http://127.0.0.1:{port}/metrics")
        if code != 200:
            return None
        out = {"rows": {}, "up": {}, "reason": {}, "stale": {}, "lane": {}, "t": time.monotonic()}
        for s in parse_text(body):
            d = s.label_dict()
            if s.name == "rocmdash_sampler_samples_total" and d.get("source") == "counter":
                out["rows"][d["gpu_id"]] = s.value
            elif s.name == "rocmdash_counter_source_up":
                out["up"][d["gpu_id"]] = s.value
            elif s.name == "rocmdash_counter_source_down_info":
                out["reason"][d["gpu_id"]] = d["reason"]
            elif s.name == "rocmdash_source_stale" and d.get("source") == "counter":
                out["stale"][d["gpu_id"]] = s.value
            elif s.name == "rocmdash_counter_source_lane":
                out["lane"][d["gpu_id"]] = s.value
        return out

    hist, codes = [], []
    try:
        deadline = time.monotonic() + 120
        while time.monotonic() < deadline:
            s = scrape()
            if s and len(s["rows"]) == 3 and len(s["up"]) == 3:
                hist.append(s)
                codes.append(get(f"http://127.0.0.1:{port}/healthz")[0])
                # done once GPU 1 went down and came back on a fresh lane with new rows
                down = [h for h in hist if h["up"].get("1") == 0.0]
                if down and s["up"]["1"] == 1.0 and s["lane"].get("1", 0) >= 1 and \
                        s["rows"]["1"] > down[-1]["rows"]["1"] + 50:
                    break
            time.sleep(0.2)
    finally:
        stop_node(p)
    log = (tmp_path / "node.log").read_text()
    down = [h for h in hist if h["up"].get("1") == 0.0]
    assert down, log[-3000:]
    assert "stalled" in down[0]["reason"]["1"], down[0]
    assert hist[-1]["up"]["1"] == 1.0 and hist[-1]["lane"]["1"] >= 1, (hist[-1], log[-3000:])
    # GPU 1's counter series were flagged stale while it was down
    assert any(h["stale"].get("1") == 1.0 for h in down), [h["stale"] for h in down]
    # flagged within 1 s of its last row: the first "down" scrape is at most ~1 s after the
    # last scrape in which GPU 1's rows still advanced
    last_adv = max(i for i in range(1, len(hist)) if hist[i]["rows"]["1"] > hist[i - 1]["rows"]["1"]
                   and hist[i]["t"] < down[0]["t"])
    assert down[0]["t"] - hist[last_adv]["t"] < 1.0 + 0.5, (down[0]["t"] - hist[last_adv]["t"])
    # GPUs 0 and 2: ~100 rows/s in every 2 s window, through the hang and the fresh lane
    for g in ("0", "2"):
        i = 0
        while i < len(hist):
            j = next((k for k in range(i, len(hist)) if hist[k]["t"] - hist[i]["t"] >= 2.0), None)
            if j is None:
                break
            rate = (hist[j]["rows"][g] - hist[i]["rows"][g]) / (hist[j]["t"] - hist[i]["t"])
            assert 60 < rate < 140, (g, i, rate)
            i = j
    assert set(codes) == {200}, codes
