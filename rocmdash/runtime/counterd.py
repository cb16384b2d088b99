"""The node's ONE device-counter process.

    python -m rocmdash.runtime.counterd --dir /dev/shm/rocmdash-<port> --devices 0,1,...,7 [--hz 100]

rocprofiler-sdk's device counting keeps one runtime thread busy-polling its completion
signal for the whole life of a counting context (rocmdash/runtime/threads.py, BASELINE.md
"counter context stopped between reads - rejected"). With one context per rank process
that is one busy core per GPU, ~8 per node. This process owns EVERY GPU's counting
context instead - one poller per node - and publishes each GPU's counter rows (MFMA
busy, HBM read / write bandwidth, GFX busy, CU active; csrc/counters.cpp) at the counter
rate into a shared-memory ring per GPU (csrc/shm_ring.h, ``ShmPublisher``: one native
thread - a LANE - per GPU, every lane reading at the same instants). The ranks' agents
read their GPU's ring (``GpuAgent(counters="node")``, ``ShmSource``) and never configure
counting.

The node supervisor (rocmdash.runtime.supervisor) starts it before the ranks and restarts
it if it dies or stalls as a whole. One GPU whose read blocks stops only its own lane:
the supervisor sees that ring's heartbeat stall (rocmdash.runtime.lanes.LaneWatch),
reports the GPU's counter source down, and after a backoff asks - through
``<dir>/control.json`` - for a fresh lane, which this process starts with a new source
and a new ring (``ShmPublisher.replace``). A rank whose ring stops advancing counts
failed reads and its counter series go stale (a metric), the SMU-table series go on.

``ROCMDASH_FAULT=ctrhang:<device>:<seconds>[:always]`` (tests) makes that device's
first lane - or, with ``always``, every lane - block in its reads after that many
seconds.

Reference anchor: the reference's own samples come from an external exporter and cost
the node nothing (/root/reference/app.py:167-176).
"""

from __future__ import annotations

import argparse
import json
import logging
import os
import signal
import threading
import time

log = logging.getLogger("rocmdash.counterd")


def ring_path(directory: str, device: int) -> str:
    """The shared-memory ring of the GPU that is HIP device ``device``."""
    return os.path.join(directory, f"ctr-dev{int(device)}.ring")


def hang_plan(devices) -> dict:
    """``ROCMDASH_FAULT=ctrhang:<device>:<seconds>[:always]`` -> {device: (seconds,
    always)} for the devices of this process; other faults (the ranks') -> {}."""
    spec = os.environ.get("ROCMDASH_FAULT", "")
    parts = spec.split(":")
    if not spec or parts[0] != "ctrhang":
        return {}
    if len(parts) not in (3, 4) or (len(parts) == 4 and parts[3] != "always"):
        raise ValueError(f"ROCMDASH_FAULT: cannot parse {spec!r}")
    dev = int(parts[1])
    return {dev: (float(parts[2]), len(parts) == 4)} if dev in devices else {}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--dir", required=True, help="directory of the per-GPU rings (tmpfs, e.g. /dev/shm/...)")
    ap.add_argument("--devices", required=True, help="HIP device index of every GPU, comma separated")
    ap.add_argument("--hz", type=float, default=float(os.environ.get("ROCMDASH_COUNTER_HZ", "100")))
    ap.add_argument("--source", default="hw", choices=["hw", "synthetic"])
    ap.add_argument("--status-s", type=float, default=10.0, help="write status.json this often")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(message)s")
    devices = sorted({int(x) for x in args.devices.split(",") if x.strip()})
    os.makedirs(args.dir, exist_ok=True)

    from . import native

    nat = native.load(with_torch=False)  # no torch in this process: ~250 MiB less per node
    hangs = hang_plan(devices)
    bdfs = {}

    def make_source(d: int, lane: int):
        if args.source == "hw":
            src = nat.make_counter_source_all(bdfs[d], d)
        else:
            src = nat.make_synthetic_source("counter", 0x5EED + 7919 * d + 104729 * lane)
        if d in hangs and (lane == 0 or hangs[d][1]):
            log.warning("fault injection: device %d lane %d hangs after %g s", d, lane, hangs[d][0])
            src = nat.make_hanging_source(src, hangs[d][0])
        return src

    if args.source == "hw":
        ok, status = native.enable_counters()  # every GPU: before the HIP runtime starts
        if not ok:
            log.error("device counting unavailable: %s", status)
            return 3
        bdfs = {d: int(nat.hip_device_bdf(d)) for d in devices}
        sources = [make_source(d, 0) for d in devices]
        from .placement import restore_affinity

        restore_affinity()
        from .threads import demote_runtime_spinners

        # the one poller of the node: demoted to SCHED_IDLE as in the per-rank service
        demoted = demote_runtime_spinners()
    else:
        sources = [make_source(d, 0) for d in devices]
        demoted = []
    paths = [ring_path(args.dir, d) for d in devices]
    pub = nat.ShmPublisher(paths, sources, args.hz)
    pub.start()
    log.info("publishing %s counters of %d GPU(s) at %g Hz into %s, one lane per GPU (SCHED_IDLE: %s)",
             args.source, len(devices), args.hz, args.dir, demoted)

    from .lanes import read_control

    stop = threading.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda *_: stop.set())
    status_path = os.path.join(args.dir, "status.json")
    t0, c0 = time.monotonic(), time.process_time()
    t_status = -1e9
    lane_gen = {d: 0 for d in devices}
    while not stop.is_set():
        # fresh lanes the supervisor asked for (a GPU whose reads stalled)
        for d, gen in read_control(args.dir).items():
            if d in lane_gen and gen > lane_gen[d]:
                try:
                    lane_gen[d] = int(pub.replace(devices.index(d), make_source(d, gen)))
                    log.info("device %d: fresh counter lane %d (asked for %d)", d, lane_gen[d], gen)
                except (RuntimeError, ValueError) as exc:
                    log.error("device %d: no fresh counter lane: %s", d, exc)
                    lane_gen[d] = gen  # asked again only with a newer generation
        now = time.monotonic()
        if now - t_status >= args.status_s:
            t_status = now
            st = pub.stats()
            doc = {"pid": os.getpid(), "devices": devices, "hz": args.hz, "source": args.source,
                   "uptime_s": round(now - t0, 1),
                   "cpu_seconds": round(time.process_time() - c0, 3),
                   "rings": [{"device": d, "path": p, "samples": int(s[0]), "failures": int(s[1]),
                              "mean_read_us": round(s[2], 2), "beat_age_s": s[4], "lane": int(s[5]),
                              "in_read_s": round(s[6], 3)} for d, p, s in zip(devices, paths, st)]}
            tmp = status_path + ".tmp"
            with open(tmp, "w") as f:
                json.dump(doc, f)
            os.replace(tmp, status_path)
        stop.wait(0.1)
    pub.stop(2.0)  # a lane blocked in a read is left behind; the process exit ends it
    log.info("stopped: %s", pub.stats())
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
