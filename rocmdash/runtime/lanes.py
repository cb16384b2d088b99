"""Per-GPU failure isolation of the node's counter process.

The node counter process (``rocmdash.runtime.counterd``) reads every GPU's device
counters on one LANE per GPU - a native thread each (``ShmPublisher``, csrc/
node_counters.cpp) - and stamps that GPU's shared-memory ring's heartbeat
(``beat_ns``, csrc/shm_ring.h) after every read. One GPU whose counter read blocks (a
reset, a hung firmware call) therefore stops only its own lane. This module is the
supervisor's side of it:

  * ``read_ring_header(path)`` reads a ring's heartbeat, producer pid and lane
    generation straight from the file (no native extension in the supervisor);
  * ``LaneWatch`` decides, from those heartbeats, which GPU's counter source is down:
    a ring whose beat is older than ``stall_s`` (5 counter periods, at least 0.25 s)
    while another GPU's beat is fresh. Such a GPU is exported as
    ``rocmdash_counter_source_up{gpu_id} 0`` with the reason; the ranks' counter series
    of that GPU go stale on their own (their ring stops advancing). After a backoff
    (``restart_delay``) the watch asks the counter process for a FRESH lane for that GPU
    (``control.json``: ``{"lanes": {device: generation}}``, which ``counterd`` applies
    with ``ShmPublisher.replace``): a new source and a new ring file, while the hung
    lane is abandoned. A lane that stalls again doubles the backoff. The other GPUs'
    lanes are never touched - no process restart, no gap in their series.

A counter process that stalls as a whole (every lane's beat old) is not a per-GPU
matter: the supervisor restarts that process (``whole_process_stalled``).

Reference anchor: in the reference each GPU's series stand alone - every result row is
parsed on its own and a missing GPU simply drops out (/root/reference/app.py:183-201,
335).
"""

from __future__ import annotations

import json
import os
import struct
import time
from dataclasses import dataclass

# offsets of csrc/shm_ring.h's ShmRingHeader words (static_assert'ed there)
RING_HEADER_OFFSETS = {"magic": 0, "producer_pid": 40, "lane": 44, "head": 128, "beat_ns": 256, "failures": 264}
RING_MAGIC = 0x31474E5248534452  # "RDSHRNG1"


def read_ring_header(path: str) -> dict | None:
    """{"pid", "lane", "head", "beat_ns", "failures"} of a counter ring, or None when the
    file is missing or not a ring. Torn reads of the 8-byte words cannot happen on
    x86-64 (aligned), and a stale value only delays a decision by one poll."""
    try:
        fd = os.open(path, os.O_RDONLY)
    except OSError:
        return None
    try:
        buf = os.pread(fd, 280, 0)
    except OSError:
        return None
    finally:
        os.close(fd)
    if len(buf) < 280:
        return None
    o = RING_HEADER_OFFSETS
    if struct.unpack_from("<Q", buf, o["magic"])[0] != RING_MAGIC:
        return None
    return {"pid": struct.unpack_from("<i", buf, o["producer_pid"])[0],
            "lane": struct.unpack_from("<i", buf, o["lane"])[0],
            "head": struct.unpack_from("<Q", buf, o["head"])[0],
            "beat_ns": struct.unpack_from("<Q", buf, o["beat_ns"])[0],
            "failures": struct.unpack_from("<Q", buf, o["failures"])[0]}


def control_path(directory: str) -> str:
    return os.path.join(directory, "control.json")


def write_control(directory: str, lanes: dict) -> None:
    """Ask the counter process for lane generations ``{device: generation}`` (atomic)."""
    path = control_path(directory)
    tmp = f"{path}.tmp.{os.getpid()}"
    with open(tmp, "w") as f:
        json.dump({"lanes": {str(int(d)): int(g) for d, g in lanes.items()}}, f)
    os.replace(tmp, path)


def read_control(directory: str) -> dict:
    """``{device: generation}`` the supervisor asked for (empty when none)."""
    try:
        with open(control_path(directory)) as f:
            doc = json.load(f)
        return {int(d): int(g) for d, g in (doc.get("lanes") or {}).items()}
    except (OSError, ValueError, AttributeError, TypeError):
        return {}


@dataclass
class LaneState:
    device: int
    up: bool = True
    reason: str = ""
    failures: int = 0  # consecutive stalls (sets the backoff)
    next_try: float = 0.0
    requested: int = 0  # lane generation asked for
    t_request: float | None = None
    readmissions: int = 0
    stalls: int = 0
    t_up: float | None = None
    age_s: float | None = None
    lane: int = 0
    pid: int = 0
    seen_key: tuple | None = None  # (pid, lane) of a ring first seen without a beat
    t_seen: float = 0.0


class LaneWatch:
    """The supervisor's per-GPU view of the counter process's lanes (see the module
    docstring). ``update(now, headers)`` takes ``{device: read_ring_header(...) or
    None}`` and returns the lane generations to request (``{device: gen}``) when that
    changed, else None. Clock: ``now`` is monotonic seconds; ``beat_ns`` is
    CLOCK_REALTIME, compared with ``wall_ns`` (defaults to ``time.time_ns()``)."""

    def __init__(self, devices, hz: float, base_s: float = 5.0, max_s: float = 300.0,
                 healthy_reset_s: float = 600.0, stall_s: float | None = None):
        from .supervisor import restart_delay

        self._delay = restart_delay
        self.hz = float(hz)
        self.stall_s = float(stall_s if stall_s is not None else max(5.0 / self.hz, 0.25))
        self.base_s, self.max_s, self.healthy_reset_s = float(base_s), float(max_s), float(healthy_reset_s)
        self.lanes = {int(d): LaneState(int(d)) for d in devices}
        self.events: list = []
        self._pid = None

    def _event(self, text: str) -> None:
        self.events.append((time.time(), text))
        del self.events[:-100]

    def ages(self, now: float, headers: dict, wall_ns: int) -> dict:
        """{device: beat age in seconds, or None while undecidable} - a lane asked for
        that never beat yet is as old as the request."""
        out = {}
        for d, st in self.lanes.items():
            h = headers.get(d)
            if h is None:
                out[d] = None
                continue
            if h["beat_ns"]:
                out[d] = max(0.0, (wall_ns - h["beat_ns"]) * 1e-9)
                continue
            # a lane that never finished a read: as old as the time its ring was first seen
            key = (h["pid"], h["lane"])
            if st.seen_key != key:
                st.seen_key, st.t_seen = key, now
            t0 = st.t_seen if st.t_request is None or h["lane"] < st.requested else max(st.t_seen, st.t_request)
            out[d] = now - t0
        return out

    def update(self, now: float, headers: dict, wall_ns: int | None = None) -> dict | None:
        wall_ns = time.time_ns() if wall_ns is None else int(wall_ns)
        pids = {h["pid"] for h in headers.values() if h is not None}
        changed = False
        if len(pids) == 1 and self._pid is not None and pids != {self._pid}:
            # the counter process started again: its lanes begin at generation 0
            for st in self.lanes.values():
                if st.requested:
                    st.requested, st.t_request, changed = 0, None, True
        if len(pids) == 1:
            self._pid = next(iter(pids))
        elif len(pids) > 1:
            # a restarted counter process is replacing the rings (the dead one's stay until
            # renamed over): no per-GPU judgement until every ring is the new process's
            return {d: st.requested for d, st in self.lanes.items() if st.requested} if changed else None
        ages = self.ages(now, headers, wall_ns)
        # evidence that the process as a whole works: lanes that actually beat recently
        fresh = [d for d, a in ages.items() if a is not None and a <= self.stall_s and headers[d]["beat_ns"]]
        for d, st in self.lanes.items():
            a = ages[d]
            h = headers.get(d)
            st.age_s = a
            st.lane = h["lane"] if h else st.lane
            st.pid = h["pid"] if h else st.pid
            if a is None:
                continue
            stalled = a > self.stall_s
            others_fresh = any(x != d for x in fresh) or len(self.lanes) == 1
            if st.up:
                if st.failures and st.t_up is not None and now - st.t_up >= self.healthy_reset_s:
                    st.failures = 0
                if stalled and others_fresh:
                    st.up = False
                    st.failures += 1
                    st.stalls += 1
                    st.reason = (f"counter reads of device {d} stalled for {a:.2f} s (lane {st.lane}) while the "
                                 f"other GPUs' lanes advanced")
                    st.next_try = now + self._delay(st.failures, self.base_s, self.max_s)
                    self._event(f"counter lane of device {d} down: {st.reason}; fresh lane in "
                                f"{st.next_try - now:.1f} s")
                continue
            # down
            if not stalled and h is not None and h["beat_ns"] and h["lane"] >= st.requested:
                st.up, st.t_up, st.reason, st.t_request = True, now, "", None
                self._event(f"counter lane of device {d} up again (lane {st.lane})")
                continue
            if st.t_request is not None and h is not None and h["lane"] >= st.requested and stalled:
                # the fresh lane stalled too: back off further
                st.failures += 1
                st.stalls += 1
                st.t_request = None
                st.reason = f"counter reads of device {d} stalled again on lane {st.lane} ({a:.2f} s)"
                st.next_try = now + self._delay(st.failures, self.base_s, self.max_s)
                self._event(f"{st.reason}; next lane in {st.next_try - now:.1f} s")
                continue
            if st.t_request is None and now >= st.next_try:
                st.requested = max(st.requested, st.lane) + 1
                st.t_request = now
                st.readmissions += 1
                changed = True
                self._event(f"counter lane of device {d}: asking for lane {st.requested}")
        if changed:
            return {d: st.requested for d, st in self.lanes.items() if st.requested}
        return None

    def whole_process_stalled(self, now: float, headers: dict, limit_s: float, wall_ns: int | None = None) -> bool:
        """Every lane's beat older than ``limit_s``: the process itself is wedged."""
        wall_ns = time.time_ns() if wall_ns is None else int(wall_ns)
        ages = self.ages(now, headers, wall_ns)
        vals = [a for a in ages.values() if a is not None]
        return bool(vals) and len(vals) == len(ages) and min(vals) > limit_s

    def down(self) -> dict:
        """{device: reason} of the lanes that are down."""
        return {d: st.reason for d, st in self.lanes.items() if not st.up}
