"""Rank-per-GPU node service: background sampling on every rank, periodic RCCL
all-gather of the window statistics, rank 0 serves ``/metrics`` (and a frame file).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \\
        --master-addr 127.0.0.1 --master-port 29511 -m rocmdash.serve --port 9400

Every rank owns its GPU's samplers (amd-smi 10 Hz, device counters 100 Hz) and
device window; every ``1 / --refresh-hz`` seconds all ranks enqueue their stats
launch and ONE ``ncclAllGather`` (RCCL over xGMI, on the process's one RCCL
communicator - the same native path bench.py measures, its first gathers validated bit
for bit against the gloo control plane) builds the [N, rows, 8] node tensor; the
publish kernel behind it hands the tensor to rank 0, which publishes it to the
exporter's HTTP thread (no collective ever runs off the main loop) and optionally
writes the dashboard frame JSON. Each rank's block of that gather also carries its
source health, per-XCD detail, its own footprint (HBM, RSS, CPU) and a stop vote, so
one collective per refresh is all the service needs, and every rank leaves the loop
after the same refresh once any rank votes to stop (SIGTERM / SIGINT, --max-refreshes).

Failure handling (the reference only wraps its fetch in one
``try/except`` -> ``st.error``, ``app.py:155, 225-227``):
  * every collective is bounded by ``--collective-timeout``: a rank that dies or hangs
    makes the others fail out of the all-gather instead of blocking forever;
  * a failed collective ends the process with exit code 3; the launcher
    (``torchrun --max-restarts``, deploy/k8s/exporter-daemonset.yaml) then tears the
    group down and starts it again, which re-creates the RCCL communicator;
  * rank 0's ``/healthz`` answers 503 once the refresh loop has not completed a
    refresh for ``--stall-seconds`` (liveness probe -> container restart);
  * every rank appends its sources' health rows to the stats it gathers, so rank 0
    exports ``rocmdash_source_stale`` / ``rocmdash_sample_age_seconds`` /
    ``rocmdash_sampler_*_total`` for EVERY GPU, and ``/healthz`` answers 503 while
    any rank's source is stale (a rank whose sampler stalls keeps answering
    collectives, so only its health rows reveal it);
  * ``ROCMDASH_FAULT=exit:<rank>:<n>`` / ``hang:<rank>:<n>`` / ``stall:<rank>:<n>``
    injects a rank loss, a hung rank, or a rank whose samplers stop (the rank keeps
    refreshing) after n refreshes, on the first launch attempt only (tests).

BASELINE.json config #3 ("8xMI355X whole-node panel via RCCL all-gather").
"""

from __future__ import annotations

import argparse
import logging
import os
import signal
import threading
import time

import numpy as np

log = logging.getLogger("rocmdash.serve")


EXIT_COLLECTIVE_FAILED = 3


class _Latest:
    def __init__(self, stall_s: float = 30.0):
        self.lock = threading.Lock()
        self.snapshot = None
        self.extra = None
        self.stall_s = stall_s
        self.t_set = time.monotonic()

    def set(self, snap, extra):
        with self.lock:
            self.snapshot, self.extra = snap, extra
            self.t_set = time.monotonic()

    def health(self):
        """(ok, message): not ok only when the refresh loop stalled. A stale source (a
        GPU's newest sample older than stale_periods of its periods: per-rank health rows,
        rocmdash.models.health) is data - ``rocmdash_source_stale`` in /metrics, named in
        the message - never a reason for the liveness probe to restart the node's
        exporter (which would take every healthy GPU's metrics down with it)."""
        with self.lock:
            age = time.monotonic() - self.t_set
            if self.snapshot is None:
                return age < self.stall_s, f"no refresh yet ({age:.1f} s since start)"
            if age >= self.stall_s:
                return False, f"last refresh {age:.2f} s ago"
            h = self.snapshot.source_health
            stale = [] if h is None else [s for s in h.statuses() if s.stale]
            msg = f"last refresh {age:.2f} s ago"
            if stale:
                ids = self.snapshot.gpu_ids
                msg += "; stale sources (see rocmdash_source_stale): " + ", ".join(
                    f"gpu {ids[s.gpu]} {s.kind}" for s in stale)
            return True, msg

    def collect(self):
        with self.lock:
            if self.snapshot is None:
                raise RuntimeError("no refresh yet")
            return self.snapshot, self.extra

    def close(self):
        pass


def _fault_plan():
    """``ROCMDASH_FAULT=<kind>:<rank>:<after>[:always]`` -> (kind, rank, after), or None.
    kinds: exit / hang / stall after ``after`` refreshes, startfail (the rank exits while
    it builds its GPU agent: a GPU whose HIP device refuses). Under the node supervisor
    ``rank`` is the GPU slot. The fault fires on the first launch attempt only
    (TORCHELASTIC_RESTART_COUNT / ROCMDASH_INCARNATION 0 or unset), or on EVERY attempt
    with ``:always`` (a GPU that stays broken)."""
    spec = os.environ.get("ROCMDASH_FAULT", "")
    if not spec or spec.startswith("ctrhang:"):  # the node counter process's fault (counterd)
        return None
    parts = spec.split(":")
    always = len(parts) == 4 and parts[3] == "always"
    if len(parts) not in (3, 4) or (len(parts) == 4 and not always):
        raise ValueError(f"ROCMDASH_FAULT: cannot parse {spec!r}")
    attempt = os.environ.get("ROCMDASH_INCARNATION", os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")) or "0"
    if attempt != "0" and not always:
        return None
    kind, rank, after = parts[:3]
    if kind not in ("exit", "hang", "stall", "startfail"):
        raise ValueError(f"ROCMDASH_FAULT: unknown fault {kind!r}")
    return kind, int(rank), int(after)


def _inject(plan, rank: int, n: int, agent=None) -> None:
    if plan is None or plan[1] != rank or n != plan[2] or plan[0] == "startfail":
        return
    log.warning("fault injection: rank %d %s after %d refreshes", rank, plan[0], n)
    if plan[0] == "stall":  # the sources stop; the rank goes on refreshing its window
        agent.stop()
        return
    if plan[0] == "exit":
        os._exit(17)
    signal.signal(signal.SIGTERM, signal.SIG_DFL)  # the launcher's teardown still ends it
    while True:  # hang: stop answering collectives, stay alive
        time.sleep(3600)


def _export_self(extra, pipe, gpu_ids) -> None:
    """Every rank's own footprint and gather state, from the control rows of the
    refresh's gather (schema.CONTROL_FIELDS, rocmdash.runtime.footprint)."""
    from .runtime.footprint import decode_control

    ctl = pipe.last_control
    if ctl is None or len(ctl) != len(gpu_ids):
        return
    rep = pipe.gather_report()
    for gid, row in zip(gpu_ids, ctl):
        d = decode_control(row)
        lab = {"gpu_id": gid}
        if d["hbm_bytes"] is not None:
            extra.add("rocmdash_self_hbm_bytes", d["hbm_bytes"], lab,
                      "Device memory (HBM) held by this GPU's rocmdash rank process (KFD per-process accounting where the "
                      "kernel exposes it, else the device's VRAM growth across the rank's start-up stages)")
        if d["rss_bytes"] is not None:
            extra.add("rocmdash_self_rss_bytes", d["rss_bytes"], lab, "Resident host memory of this GPU's rocmdash rank")
        if d["cpu_seconds"] is not None:
            idle = d["cpu_idle_seconds"] or 0.0
            h = ("CPU seconds used by this GPU's rocmdash rank (all threads), by scheduling class: idle = SCHED_IDLE "
                 "threads (the runtime's demoted busy-poller, rocmdash.runtime.threads), normal = the rest")
            extra.add("rocmdash_self_cpu_seconds_total", max(0.0, d["cpu_seconds"] - idle), dict(lab, **{"class": "normal"}),
                      h, "counter")
            extra.add("rocmdash_self_cpu_seconds_total", idle, dict(lab, **{"class": "idle"}), h, "counter")
        if d["native_gather"] is not None:
            extra.add("rocmdash_gather_native", d["native_gather"], lab,
                      "1 when the rank gathers with the native RCCL ncclAllGather, 0 on the host fallback")
        if d["gather_validated"] is not None:
            extra.add("rocmdash_gather_validated", d["gather_validated"], lab,
                      "Native gathers checked bit for bit against the control-plane gather at start-up")
    _export_sources(extra, pipe, gpu_ids)
    extra.add("rocmdash_gather_validate_target", rep["validate_target"], {},
              "Native gathers each rank checks bit for bit at start-up (0: not on the native path)")
    fp = pipe.footprint
    for stage, rec in (fp.stages.items() if fp is not None else ()):
        if rec.get("hbm") is not None:
            extra.add("rocmdash_self_hbm_stage_bytes", rec["hbm"], {"gpu_id": gpu_ids[0], "stage": stage},
                      "Rank 0's process HBM after each start-up stage (start, agent, pipeline + RCCL, ...)")


def _export_sources(extra, pipe, gpu_ids) -> None:
    """Every rank's amd-smi fast-path state from the source rows of the refresh's gather
    (schema.SOURCE_FIELDS): raw SMU table or amd-smi, and its calibration - which
    retries a refusal every ROCMDASH_SMI_RECALIBRATE_S (csrc/sources.h
    RawCalibrationPolicy). Rank 0's calibration text goes out as an info series."""
    import math

    from .models.schema import SOURCE_INDEX

    src = pipe.last_source
    if src is None or len(src) != len(gpu_ids):
        return
    for gid, row in zip(gpu_ids, src):
        lab = {"gpu_id": gid}
        v = float(row[SOURCE_INDEX["smi_raw_path"]])
        if math.isnan(v):
            continue  # not an amd-smi source (synthetic / replay)
        extra.add("rocmdash_smi_raw_path", v, lab,
                  "1 when this GPU's SMU metrics table is read raw from sysfs (calibrated against amd-smi), 0 on the "
                  "amd-smi library path")
        extra.add("rocmdash_smi_calibration_attempts_total", row[SOURCE_INDEX["smi_calibration_attempts"]], lab,
                  "Raw SMU-table calibration attempts (start-up + retries after a refusal)", "counter")
        extra.add("rocmdash_smi_calibration_matched", row[SOURCE_INDEX["smi_calibration_matched"]], lab,
                  "Raw / amd-smi / raw triples that decoded the same values in the last calibration attempt (of 8; "
                  ">= 6 turns the raw path on)")
        extra.add("rocmdash_smi_calibration_promotions_total", row[SOURCE_INDEX["smi_calibration_promotions"]], lab,
                  "Times a calibration retry promoted this GPU's source to the raw path", "counter")
    cal = pipe.agent.info_calibration() if hasattr(pipe.agent, "info_calibration") else None
    if cal:
        extra.add("rocmdash_smi_calibration_info", 1.0, {"gpu_id": gpu_ids[0], "calibration": cal},
                  "Rank 0's last raw SMU-table calibration result (text)")


def refresh_node(pipe, agg, nws, latest, frame_out=None):
    """One service refresh on every rank (collective). ONE gather carries every rank's
    stats, source health, per-XCD detail, footprint and stop vote (+ the node-window
    gather with ``nws``); rank 0 hands the snapshot and the service's own metrics to
    ``latest`` (the exporter's HTTP thread reads it) and optionally writes the frame.
    Returns every rank's stop vote. Raises when a collective fails (a rank is gone)."""
    from .prom.exposition import Exposition
    from .viz.panels import render_frame_json

    t0 = time.perf_counter()
    snap = pipe.latest_snapshot()
    node_stats = nws.refresh() if nws is not None else None  # collective too
    votes = pipe.stop_votes()
    t1 = time.perf_counter()
    wall1 = time.time()
    if pipe.is_root:
        extra = Exposition()
        extra.add("rocmdash_node_refresh_seconds", t1 - t0, {}, "Stats launch + RCCL all-gather + hand-off of the last refresh")
        # wall clock of that refresh: with rocmdash_sample_age_seconds (age at the
        # refresh) a reader gets every sample's own time, hence its age on display
        extra.add("rocmdash_node_refresh_timestamp_seconds", wall1, {},
                  "Unix time the last node refresh completed (sample time = this - rocmdash_sample_age_seconds)")
        extra.add("rocmdash_node_ranks", agg.world_size, {}, "Ranks (GPUs) in the node communicator")
        for stage, sec in pipe.stage_seconds().items():
            extra.add("rocmdash_stage_seconds", sec, {"stage": stage},
                      "One stage of the last refresh on rank 0: stats_kernel (span between HIP events recorded "
                      "right before and after the window-stats launch call - on an idle GPU it includes the "
                      "host's launch call, not only the kernel), stats_launch_host (that launch call's host "
                      "time), side_rows_h2d (health / footprint rows from pinned memory), allgather (native "
                      "RCCL ncclAllGather, incl. the wait for the slowest rank), publish (hand-off kernel); "
                      "the last three are device time between HIP events")
        _export_self(extra, pipe, snap.gpu_ids)
        if node_stats is not None:
            snap.node_window = node_stats.cpu().numpy().astype("float64")
        latest.set(snap, extra)
        if frame_out:
            payload = render_frame_json(snap, snap.gpu_ids, extended=True)
            tmp = frame_out + ".tmp"
            with open(tmp, "w") as f:
                f.write(payload)
            os.replace(tmp, frame_out)
    return votes


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
    ap.add_argument("--collective-timeout", type=float,
                    default=float(os.environ.get("ROCMDASH_COLLECTIVE_TIMEOUT", "60")),
                    help="seconds a collective may wait for a silent rank before the service exits for a restart")
    ap.add_argument("--node-window", action="store_true",
                    help="also export node-wide window statistics (all GPUs' windows, one extra all-gather)")
    ap.add_argument("--stall-seconds", type=float, default=0.0,
                    help="/healthz turns 503 after this long without a refresh (default: max(10 s, 5 periods))")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(message)s")

    from .parallel.membership import Membership

    mem = Membership.from_environ(args.collective_timeout)
    if mem is not None:  # started by the node supervisor (rocmdash.launch)
        return main_supervised(args, mem)

    from .runtime import native

    native.load()
    from .parallel.node import device_index_for
    from .runtime.footprint import Footprint
    from .runtime.topology import bdf_of_hip_device

    # the footprint's baseline: device VRAM before this process starts the HIP runtime
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    fp = Footprint(bdf=None if args.cpu else bdf_of_hip_device(device_index_for(local)))
    fp.mark("start")
    if not args.cpu and args.counters in ("auto", "hw") and args.source != "synthetic":
        native.enable_counters()
    import torch.distributed as dist

    from .parallel.node import NodeAggregator, dist_env_from_environ
    from .prom.exporter import Exporter
    from .runtime.agent import GpuAgent
    from .runtime.pipeline import NodePipeline

    env = dist_env_from_environ(prefer_gpu=not args.cpu, timeout_s=args.collective_timeout)
    fp.device = env.device if env.device.type == "cuda" else None
    fp.mark("hip")
    agent = GpuAgent(env.device.index if env.device.type == "cuda" else env.local_rank, source=args.source,
                     counters=args.counters, use_gpu=env.device.type == "cuda")
    fp.mark("agent")
    demoted = []
    if agent.info.counter_backend == "rocprofiler":
        # the runtime's busy-poller (threads.py), identified now: the counting context
        # is the only thing spinning before the RCCL communicator (whose proxy threads
        # may poll too) exists
        from .runtime.threads import demote_runtime_spinners

        demoted = demote_runtime_spinners()
    agg = NodeAggregator()
    pipe = NodePipeline(agent, agg, device_timing=True, health=True, collective_timeout_s=args.collective_timeout)
    pipe.footprint = fp
    fp.mark("pipeline")  # + the RCCL communicator and node-tensor buffers at N > 1
    nws = None
    if args.node_window:
        from .parallel.node_window import NodeWindowStats

        nws = NodeWindowStats(agent, agg, collective_timeout_s=args.collective_timeout)
    agent.start()
    log.info("rank %d: gather %s; footprint after start-up: %s; SCHED_IDLE: %s", env.rank, pipe.gather_report(),
             {k: {kk: vv for kk, vv in v.items() if vv is not None} for k, v in fp.stages.items()}, demoted)

    stop = threading.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda *_: stop.set())

    period = 1.0 / args.refresh_hz
    latest = _Latest(args.stall_seconds or max(10.0, 5 * period))
    exporter = None
    if pipe.is_root:
        exporter = Exporter(latest)
        exporter.serve(args.host, args.port)
        log.info("rank 0 serving /metrics on %s:%d for %d GPU(s)", args.host, exporter.port, agg.world_size)

    fault = _fault_plan()
    n = 0
    next_t = time.monotonic()
    rc = 0
    while True:
        _inject(fault, env.rank, n, agent)
        # this rank's stop vote rides in its block of this refresh's gather
        pipe.stop_vote = 1.0 if (stop.is_set() or (args.max_refreshes and n + 1 >= args.max_refreshes)) else 0.0
        try:
            votes = refresh_node(pipe, agg, nws, latest, frame_out=args.frame_out)
            if n == 0:  # buffers the first refresh allocates (gather outputs, node window)
                fp.mark("first_refresh")
        except Exception as e:  # a rank died or hung: leave for the launcher to restart the group
            log.error("rank %d: node all-gather failed after %d refreshes (%s); exiting for a communicator restart",
                      env.rank, n, str(e).splitlines()[0] if str(e) else type(e).__name__)
            rc = EXIT_COLLECTIVE_FAILED
            break
        n += 1
        if votes is not None and float(np.nanmax(votes)) >= 1.0:  # some rank votes to stop: all leave together
            break
        next_t += period
        delay = next_t - time.monotonic()
        if delay > 0:
            stop.wait(delay)
        else:
            next_t = time.monotonic()

    agent.close()
    pipe.close()
    if exporter is not None:
        exporter.close()
    if env.initialized_here and rc == 0:  # a broken communicator is left to process exit
        dist.destroy_process_group()
    log.info("rank %d stopped after %d refreshes (exit %d)", env.rank, n, rc)
    return rc


VOTE_STOP = 1  # control-row vote bits (schema.CONTROL_INDEX["stop"]): leave and exit
VOTE_REGROUP = 2  # leave this epoch and join the supervisor's next one


def vote_flags(votes) -> int:
    """OR of every rank's vote bits carried by one gather."""
    out = 0
    for v in (() if votes is None else np.asarray(votes).ravel()):
        if v == v:
            out |= int(v)
    return out


class _PushLatest:
    """``latest`` of a supervised epoch root: each refresh's snapshot goes to the
    supervisor, which serves /metrics and /healthz (rocmdash.runtime.supervisor)."""

    def __init__(self, pusher, epoch: int):
        self.pusher = pusher
        self.epoch = epoch

    def set(self, snap, extra):
        self.pusher.push(self.epoch, snap, extra)


def _join_epoch(mem, epoch: int, members: list, timeout_s: float) -> None:
    """The control plane of one epoch: a gloo process group of its members on the
    supervisor's store (prefix ``e<epoch>/``), rank = position in the member list."""
    from datetime import timedelta

    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()
    dist.init_process_group("gloo", store=mem.pg_store(epoch), rank=members.index(mem.slot),
                            world_size=len(members), timeout=timedelta(seconds=float(timeout_s)))


def _leave_epoch(pipe, agg) -> None:
    import torch.distributed as dist

    if pipe is not None:
        pipe.close()
    if agg is not None and agg.native is not None:
        agg.native.close()  # this epoch's communicator (ncclCommAbort: a peer may be gone)
        agg.native = None
    if dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception as e:  # noqa: BLE001 - a broken group is dropped either way
            log.warning("process group teardown: %s", e)


def main_supervised(args, mem) -> int:
    """One GPU slot under the node supervisor: the agent (sources, rings, device window)
    lives as long as the process; the node refresh runs inside the epochs the supervisor
    forms (rocmdash.parallel.membership). A failed collective is reported and this rank
    waits for the next epoch - it never takes its peers down with it."""
    import torch

    from .parallel.membership import SnapshotPusher
    from .parallel.node import NodeAggregator, device_index_for, oversubscribed
    from .runtime import native
    from .runtime.footprint import Footprint
    from .runtime.topology import bdf_of_hip_device

    slot = mem.slot
    fault = _fault_plan()
    native.load()
    # device_count(), not is_available(): the latter starts the HIP runtime, and device
    # counting (enable_counters below) must be registered before it does - a one-GPU node
    # (no counter process) otherwise serves its counters as "unavailable"
    use_gpu = not args.cpu and torch.cuda.device_count() > 0
    dev_index = device_index_for(slot)
    fp = Footprint(bdf=bdf_of_hip_device(dev_index) if use_gpu else None)
    fp.mark("start")
    counters = args.counters
    if os.environ.get("ROCMDASH_COUNTER_SHM") and counters != "off":
        counters = "node"  # the node's counter process reads this GPU's counters (counterd)
    elif use_gpu and counters in ("auto", "hw") and args.source != "synthetic":
        native.enable_counters()
    if oversubscribed():  # before RCCL loads: every slot its own "host" (parallel.node.oversubscribed)
        os.environ["NCCL_HOSTID"] = f"rocmdash-virt-{slot}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    if fault is not None and fault[0] == "startfail" and fault[1] == slot:
        log.warning("fault injection: slot %d startfail (incarnation %d)", slot, mem.incarnation)
        os._exit(18)
    from .runtime.agent import GpuAgent
    from .runtime.pipeline import NodePipeline

    device = torch.device("cuda", dev_index) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
    fp.device = device if use_gpu else None
    fp.mark("hip")
    agent = GpuAgent(dev_index if use_gpu else slot, source=args.source, counters=counters, use_gpu=use_gpu)
    fp.mark("agent")
    if agent.info.counter_backend == "rocprofiler":
        from .runtime.threads import demote_runtime_spinners

        demote_runtime_spinners()
    agent.start()
    mem.announce_ready(dict(agent.info.as_dict(), slot=slot, incarnation=mem.incarnation, pid=os.getpid()))
    log.info("slot %d (incarnation %d): agent ready on %s", slot, mem.incarnation, device)

    stop = threading.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda *_: stop.set())
    pusher = SnapshotPusher()
    period = 1.0 / args.refresh_hz
    n = 0  # refreshes this process took part in (all epochs)
    leaving = False
    while not leaving and not stop.is_set():
        got = mem.wait_epoch(stop)
        if got is None:
            break
        epoch, members = got
        pipe = agg = nws = None
        try:
            _join_epoch(mem, epoch, members, args.collective_timeout)
            agg = NodeAggregator()
            agg.abandon = mem.newer_epoch
            pipe = NodePipeline(agent, agg, device_timing=True, health=True, collective_timeout_s=args.collective_timeout,
                                rank_labels=list(members))
            pipe.footprint = fp
            if args.node_window:
                from .parallel.node_window import NodeWindowStats

                nws = NodeWindowStats(agent, agg, collective_timeout_s=args.collective_timeout)
        except Exception as e:  # noqa: BLE001 - a member that never joined: reported, next epoch
            log.error("slot %d: joining epoch %d failed (%s)", slot, epoch, str(e).splitlines()[0] if str(e) else e)
            mem.report_failure(epoch, f"join: {e}")
            _leave_epoch(pipe, agg)
            continue
        latest = _PushLatest(pusher, epoch) if pipe.is_root else None
        log.info("slot %d: epoch %d rank %d of %d (members %s); gather %s", slot, epoch, agg.rank, agg.world_size,
                 members, pipe.gather_report()["status"])
        next_t = time.monotonic()
        while True:
            _inject(fault, slot, n, agent)
            flags = 0
            if stop.is_set() or (args.max_refreshes and n + 1 >= args.max_refreshes):
                flags |= VOTE_STOP
            if pipe.is_root and mem.newer_epoch():
                flags |= VOTE_REGROUP
            pipe.stop_vote = float(flags)
            try:
                votes = refresh_node(pipe, agg, nws, latest, frame_out=args.frame_out)
                if n == 0:
                    fp.mark("first_refresh")
            except Exception as e:  # noqa: BLE001 - a member is gone or hung
                msg = str(e).splitlines()[0] if str(e) else type(e).__name__
                log.error("slot %d: epoch %d refresh failed after %d refreshes (%s); waiting for the next epoch",
                          slot, epoch, n, msg)
                if not mem.newer_epoch():
                    mem.report_failure(epoch, msg)
                break
            n += 1
            v = vote_flags(votes)
            if v & VOTE_STOP:
                leaving = True
                break
            if v & VOTE_REGROUP:
                break
            next_t += period
            delay = next_t - time.monotonic()
            if delay > 0:
                stop.wait(delay)
            else:
                next_t = time.monotonic()
        _leave_epoch(pipe, agg)
        nws = None
    agent.close()
    pusher.close()
    if leaving or stop.is_set():
        mem.announce_stopped()
    log.info("slot %d stopped after %d refreshes", slot, n)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
