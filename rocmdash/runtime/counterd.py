"""The node's ONE device-counter process.

    python -m rocmdash.runtime.counterd --dir /dev/shm/rocmdash-<port> --devices 0,1,...,7 [--hz 100]

rocprofiler-sdk's device counting keeps one runtime thread busy-polling its completion
signal for the whole life of a counting context (rocmdash/runtime/threads.py, BASELINE.md
"counter context stopped between reads - rejected"). With one context per rank process
that is one busy core per GPU, ~8 per node. This process owns EVERY GPU's counting
context instead - one poller per node - and publishes each GPU's counter rows (MFMA
busy, HBM read / write bandwidth, GFX busy, CU active; csrc/counters.cpp) at the counter
rate into a shared-memory ring per GPU (csrc/shm_ring.h, ``ShmPublisher``: one native
thread, reads back to back over the GPUs each period). The ranks' agents read their
GPU's ring (``GpuAgent(counters="node")``, ``ShmSource``) and never configure counting.

The node supervisor (rocmdash.runtime.supervisor) starts it before the ranks and restarts
it if it dies; a rank whose ring stops advancing counts failed reads and its counter
series go stale (a metric), the SMU-table series go on.

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
    sources = []
    if args.source == "hw":
        ok, status = native.enable_counters()  # every GPU: before the HIP runtime starts
        if not ok:
            log.error("device counting unavailable: %s", status)
            return 3
        for d in devices:
            bdf = int(nat.hip_device_bdf(d))
            sources.append(nat.make_counter_source_all(bdf, d))
        from .placement import restore_affinity

        restore_affinity()
        from .threads import demote_runtime_spinners

        # the one poller of the node: demoted to SCHED_IDLE as in the per-rank service
        demoted = demote_runtime_spinners()
    else:
        sources = [nat.make_synthetic_source("counter", 0x5EED + 7919 * d) for d in devices]
        demoted = []
    paths = [ring_path(args.dir, d) for d in devices]
    pub = nat.ShmPublisher(paths, sources, args.hz)
    pub.start()
    log.info("publishing %s counters of %d GPU(s) at %g Hz into %s (SCHED_IDLE: %s)", args.source, len(devices),
             args.hz, args.dir, demoted)

    stop = threading.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda *_: stop.set())
    status_path = os.path.join(args.dir, "status.json")
    t0, c0 = time.monotonic(), time.process_time()
    while not stop.is_set():
        st = pub.stats()
        doc = {"pid": os.getpid(), "devices": devices, "hz": args.hz, "source": args.source,
               "uptime_s": round(time.monotonic() - t0, 1),
               "cpu_seconds": round(time.process_time() - c0, 3),
               "rings": [{"device": d, "path": p, "samples": int(s[0]), "failures": int(s[1]),
                          "mean_read_us": round(s[2], 2)} for d, p, s in zip(devices, paths, st)]}
        tmp = status_path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(doc, f)
        os.replace(tmp, status_path)
        stop.wait(args.status_s)
    pub.stop()
    log.info("stopped: %s", pub.stats())
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
