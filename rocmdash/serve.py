"""Rank-per-GPU node service: background sampling on every rank, periodic RCCL
all-gather of the window statistics, rank 0 serves ``/metrics`` (and a frame file).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \\
        --master-addr 127.0.0.1 --master-port 29511 -m rocmdash.serve --port 9400

Every rank owns its GPU's samplers (amd-smi 10 Hz, device counters 100 Hz) and
device window; every ``1 / --refresh-hz`` seconds all ranks enqueue their stats
launch and ONE ``all_gather_into_tensor`` (RCCL over xGMI) builds the [N, S, 8] node
tensor; rank 0 publishes it to the exporter's HTTP thread (no collective ever runs
off the main loop) and optionally writes the dashboard frame JSON. A one-element
all-reduce per refresh carries the stop flag so every rank leaves the loop together
(SIGTERM / SIGINT on any rank).

BASELINE.json config #3 ("8xMI355X whole-node panel via RCCL all-gather").
"""

from __future__ import annotations

import argparse
import logging
import os
import signal
import threading
import time

log = logging.getLogger("rocmdash.serve")


class _Latest:
    def __init__(self):
        self.lock = threading.Lock()
        self.snapshot = None
        self.extra = None

    def set(self, snap, extra):
        with self.lock:
            self.snapshot, self.extra = snap, extra

    def collect(self):
        with self.lock:
            if self.snapshot is None:
                raise RuntimeError("no refresh yet")
            return self.snapshot, self.extra

    def close(self):
        pass


def main(argv=None) -> int:
    from . import config

    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=config.EXPORTER_PORT)
    ap.add_argument("--refresh-hz", type=float, default=1.0)
    ap.add_argument("--source", default="auto", choices=["auto", "hw", "synthetic"])
    ap.add_argument("--counters", default="auto", choices=["auto", "hw", "synthetic", "off"])
    ap.add_argument("--frame-out", default=None, help="rank 0 writes the dashboard frame JSON here each refresh")
    ap.add_argument("--max-refreshes", type=int, default=0, help="stop after N refreshes (0 = run until signalled)")
    ap.add_argument("--cpu", action="store_true")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(message)s")

    from .runtime import native

    native.load()
    if not args.cpu and args.counters in ("auto", "hw") and args.source != "synthetic":
        native.enable_counters()
    import torch
    import torch.distributed as dist

    from .parallel.node import NodeAggregator, dist_env_from_environ
    from .prom.exporter import Exporter
    from .prom.exposition import Exposition
    from .runtime.agent import GpuAgent
    from .runtime.pipeline import NodePipeline
    from .viz.panels import render_frame_json

    env = dist_env_from_environ(prefer_gpu=not args.cpu)
    agent = GpuAgent(env.local_rank, source=args.source, counters=args.counters, use_gpu=env.device.type == "cuda")
    agg = NodeAggregator()
    pipe = NodePipeline(agent, agg)
    agent.start()

    stop = threading.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda *_: stop.set())

    latest = _Latest()
    exporter = None
    if pipe.is_root:
        exporter = Exporter(latest)
        exporter.serve(args.host, args.port)
        log.info("rank 0 serving /metrics on %s:%d for %d GPU(s)", args.host, exporter.port, agg.world_size)

    period = 1.0 / args.refresh_hz
    flag = torch.zeros(1, dtype=torch.int32, device=env.device if agg.backend == "nccl" else "cpu")
    n = 0
    next_t = time.monotonic()
    while True:
        t0 = time.perf_counter()
        snap = pipe.latest_snapshot()  # collective: every rank, every refresh
        t1 = time.perf_counter()
        if pipe.is_root:
            extra = Exposition()
            extra.add("rocmdash_node_refresh_seconds", t1 - t0, {}, "Stats launch + RCCL all-gather + D2H of the last refresh")
            extra.add("rocmdash_node_ranks", agg.world_size, {}, "Ranks (GPUs) in the node communicator")
            latest.set(snap, extra)
            if args.frame_out:
                payload = render_frame_json(snap, snap.gpu_ids, extended=True)
                tmp = args.frame_out + ".tmp"
                with open(tmp, "w") as f:
                    f.write(payload)
                os.replace(tmp, args.frame_out)
        n += 1
        flag.fill_(1 if (stop.is_set() or (args.max_refreshes and n >= args.max_refreshes)) else 0)
        if agg.world_size > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if int(flag.item()):
            break
        next_t += period
        delay = next_t - time.monotonic()
        if delay > 0:
            stop.wait(delay)
        else:
            next_t = time.monotonic()

    agent.close()
    if exporter is not None:
        exporter.close()
    if env.initialized_here:
        dist.destroy_process_group()
    log.info("rank %d stopped after %d refreshes", env.rank, n)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
