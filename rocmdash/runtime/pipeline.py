"""The refresh pipeline of one node: per-rank agent -> RCCL all-gather -> rank-0 frame.

One ``step()`` is one dashboard refresh (BASELINE.md "full refresh"):

  1. (closed-loop mode) every rank samples its GPU's sources once -> pinned rings;
  2. every rank enqueues ONE window-stats launch on its stream; the kernel pulls the
     entering rows straight from the mapped pinned rings (hipMemcpyAsync staging only
     before a full re-sort);
  3. N > 1: ONE ``ncclAllGather`` on the same stream builds the [N, rows, 8] node tensor
     (RCCL over xGMI, rocmdash's own communicator) and the publish kernel hands it to
     rank 0's pinned buffer; N = 1: the gather is the identity and the stats kernel
     writes rank 0's pinned buffer itself (tagged words, no D2H copy);
  4. rank 0 builds the ``NodeSnapshot`` and renders the dashboard frame (4 + 4N figures
     + statistics tables) to its JSON payload - natively (csrc/frame_render.cpp,
     byte-identical to the Python frame).

The first ``ROCMDASH_GATHER_VALIDATE`` (default 8) native gathers are checked bit for
bit against the control plane's host gather on every rank; any mismatch anywhere moves
every rank to the host gather together (``gather_status``).

Reference counterpart: one iteration of ``app.py:326-486`` minus the 5 s sleep
(fetch via Prometheus ``app.py:331`` -> pandas -> Plotly figures).
"""

from __future__ import annotations

import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..models.schema import CONTROL_INDEX, CONTROL_ROWS, HEALTH_SOURCES, NUM_STATS, SOURCE_INDEX, STAT_INDEX, XCD_ROWS
from ..parallel.node import NodeAggregator
from ..utils.trace import trace_range
from ..viz.panels import CompiledFrame, NodeSnapshot, SourceHealth, render_frame_json
from .agent import GpuAgent

LAST = STAT_INDEX["last"]
# host-out refreshes wait on the stats kernel's completion flag (0: stream synchronise)
_DONE_FLAG = os.environ.get("ROCMDASH_DONE_FLAG", "1") not in ("0", "off", "false")
# host-out completion: 2 = tagged output words (default), 1 = last-workgroup flag
_HOST_SIGNAL = 1 if os.environ.get("ROCMDASH_TAGGED_OUT", "1") in ("0", "off", "false") else 2
_VALIDATE = int(os.environ.get("ROCMDASH_GATHER_VALIDATE", "8"))


@dataclass
class StepTiming:
    sample_ms: float = 0.0
    device_ms: float = 0.0  # enqueue copies + kernel + all-gather + D2H (host-observed)
    render_ms: float = 0.0
    total_ms: float = 0.0
    payload_bytes: int = 0


@dataclass
class NodePipeline:
    agent: GpuAgent
    aggregator: NodeAggregator
    selected: list | None = None  # gpu ids shown (default: all)
    use_gauge: bool = True
    extended: bool = False
    prefetch: bool = False  # sample refresh i+1 on native threads while refresh i renders
    # "closed": each refresh takes one sample per source (prefetched or inline);
    # "free": the sources read back to back on their own threads (GpuAgent.start_free)
    # and each refresh waits until every source has at least one new row, then reduces
    # all rows that arrived (start_sampling() switches the agent over)
    sampling: str = "closed"
    infos: list = field(default_factory=list)
    # rehearsal only (bench --rehearse-gpus): rank 0 renders a frame for this many GPUs
    # by repeating the gathered ones - the rank-0 render cost of a bigger node on a
    # smaller box. Never used for reported numbers.
    render_gpus: int = 0
    # record HIP events around the stats kernel and the all-gather of each gather()
    # (a few µs per refresh: the 1 Hz service turns it on, the bench does not);
    # stage_seconds() reads them once the refresh has been synchronised
    device_timing: bool = False
    # append every rank's side rows to its gathered stats - source health
    # (schema.HEALTH_FIELDS, one row per source), per-XCD busy / clocks and the rank's
    # stop vote (schema.XCD_ROWS, CONTROL_FIELDS): rank 0 then exports every GPU's
    # sampler staleness, failures and XCD detail, and every rank learns whether any
    # rank wants to stop, all from the ONE all-gather of the refresh (rocmdash.serve)
    health: bool = False
    # world size 1 without a forced collective: let the stats kernel write the pinned
    # host buffer directly (the gather is the identity). False = always gather.
    allow_host_out: bool = True
    # the node gather on the aggregator's native data-plane transport (None: whenever a
    # GPU pipeline gathers; True: also on the CPU, with a transport the caller enabled -
    # the gloo stand-in of the multi-rank tests)
    native_gather: bool | None = None
    # how long a native gather may wait for the slowest rank before the communicator is
    # aborted and the refresh fails (a rank died or hung: rocmdash.serve restarts)
    collective_timeout_s: float = field(default_factory=lambda: float(os.environ.get("ROCMDASH_COLLECTIVE_TIMEOUT", "60")))
    # labels of the ranks when their GPUs' own ids collide (synthetic sources, several
    # ranks on one GPU): default the rank numbers; the supervised service passes the
    # ranks' node slots, so a GPU keeps its label when the epoch's ranks renumber
    rank_labels: list | None = None

    def __post_init__(self):
        self._prefetch_t0 = None
        self.launch_host_s = None  # timed refreshes: host time of the stats launch (between its events)
        self._free_calls = None  # free-running: the sources' call counts at the last refresh
        self._events = None
        self._stage_host = None
        self.infos = self.aggregator.all_gather_object(self.agent.info.as_dict())
        series = {tuple(i["series"]) for i in self.infos}
        if len(series) != 1:
            raise RuntimeError(f"ranks disagree on the series layout: {series}")
        self.series = tuple(self.infos[0]["series"])
        self.gpu_ids = [i["gpu_id"] for i in self.infos]
        if len(set(self.gpu_ids)) != len(self.gpu_ids):  # e.g. synthetic sources on every rank
            labels = self.rank_labels if self.rank_labels is not None else range(len(self.infos))
            self.gpu_ids = [str(r) for r in labels]
        self.is_root = self.aggregator.rank == 0
        self._compiled = None  # CompiledFrame for the current selection (None: not built, False: n/a)
        self._compiled_sel = None
        self._host = None
        S = len(self.series)
        # health, XCD, control + source rows
        self.side = len(HEALTH_SOURCES) + XCD_ROWS + CONTROL_ROWS if self.health else 0
        self.rows = S + self.side  # rows per rank in the node tensor
        if self.agent.use_gpu and self.is_root:
            shape = (self.aggregator.world_size, self.rows, NUM_STATS)
            self._host = torch.empty(shape, dtype=torch.float32, pin_memory=True)
        # world size 1 and no forced collective: the gather is the identity, so the
        # stats kernel writes its output straight into the pinned host buffer (mapped,
        # device-accessible) - no D2H copy
        self.host_out = (self._host is not None and not self.aggregator.collective and self.allow_host_out
                         and os.environ.get("ROCMDASH_HOST_OUT", "1") != "0")
        self._local = None  # [rows, 8] on the device: stats + side rows of this rank
        self._side = None  # [side, 8] host staging of the side rows (pinned on GPUs)
        if self.health:
            pin = self.agent.use_gpu
            self._side = torch.empty((self.side, NUM_STATS), dtype=torch.float32, pin_memory=pin)
            if not self.host_out:
                self._local = torch.empty((self.rows, NUM_STATS), dtype=torch.float32, device=self.agent.device)
        # side rows of the last refresh on rank 0 (None without health): node health
        # [N, H, 8], per-XCD detail [N, 2, XCDS], control rows [N, 8] (stop vote and the
        # rank's own footprint, schema.CONTROL_FIELDS), stop votes [N]
        self.last_health = None
        self.last_xcd = None
        self.last_control = None
        self.last_source = None  # [N, 8] every rank's source row (schema.SOURCE_FIELDS)
        self.last_stop = None
        self.footprint = None  # rocmdash.runtime.footprint.Footprint of this rank (health only)
        self.stop_vote = 0.0  # this rank's vote, carried by its next gathered block
        self._node = None  # the last gathered node tensor (non-root ranks read the votes from it)
        if self.health:
            from .footprint import Footprint

            self.footprint = Footprint(self.agent.device if self.agent.use_gpu else None)
        # N > 1 (or a forced collective): the node gather is one ncclAllGather on this
        # stream, on the process's one RCCL communicator (the aggregator's data plane),
        # and a publish kernel puts the node tensor into rank 0's pinned buffer with a
        # completion signal every rank spins on - no torch collective, D2H copy or
        # stream synchronisation on the hot path (rocmdash.parallel.node.NativeNodeGather).
        # The same path runs with HIP-event timing (the service, the bench's side run).
        # If any rank cannot set it up, every rank uses the host gather instead.
        self._ng = None
        self.gather_status = "identity" if not self.aggregator.collective else "host"
        want = self.native_gather if self.native_gather is not None else self.agent.use_gpu
        if want and not self.host_out and self.aggregator.collective:
            from ..parallel.node import NativeGatherUnavailable, NativeNodeGather

            dev = self.agent.device
            if self.aggregator.enable_native(dev):
                err = None
                try:
                    self._ng = NativeNodeGather(self.aggregator, dev, (self.rows, NUM_STATS),
                                                root_host=self._host if self.is_root else None)
                except (NativeGatherUnavailable, RuntimeError, ValueError) as e:  # e.g. no mapped host memory
                    self._ng, err = None, f"rank {self.aggregator.rank}: {e}"
                # every rank gathers natively, or none does (a rank on the other path would
                # leave its peers' ncclAllGather waiting)
                errs = [e for e in self.aggregator.all_gather_object(err) if e]
                if errs:
                    self._ng = None
                    self.aggregator.native_error = "; ".join(errs)
                else:
                    self.gather_status = "native"
            if self._ng is None and self.aggregator.native_error:
                import sys

                print(f"[rocmdash] native RCCL gather unavailable ({self.aggregator.native_error}); "
                      "gathering through the control plane", file=sys.stderr, flush=True)
        self.validate_gathers = _VALIDATE if self._ng is not None else 0

    # ------------------------------------------------------------------
    def gather(self) -> torch.Tensor:
        """Steps 2-3: local stats -> node tensor (device; with ``host_out`` the pinned
        host buffer itself, valid once the stream is synchronised; after a fallback,
        possibly a host tensor)."""
        if self.device_timing:
            return self._gather_timed()
        if self.host_out:
            self._local_stats()
            return self._host
        if self._ng is not None:
            return self._native_gather(self._local_stats())
        return self._fallback_gather(self._local_stats())

    def _stream(self) -> int:
        dev = self.agent.device
        return torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0

    def _native_gather(self, local, ev=None):
        """ncclAllGather + publish on this rank's stream; HIP events between them when
        timed; the first ``validate_gathers`` are cross-checked (``_validate``)."""
        agg = self.aggregator
        agg.calls += 1
        agg.collectives += 1
        stream = self._stream()
        node = self._ng.all_gather(local, stream)
        if ev is not None:
            ev[2].record()
        self._ng.publish(stream)
        if ev is not None:
            ev[3].record()
        if self._ng.validated < self.validate_gathers:
            node = self._validate(local, node)
        return node

    def _fallback_gather(self, local):
        """The agreed fallback: through host memory on the gloo control plane (rank 0
        needs the node tensor on the host anyway), else the aggregator's collective."""
        agg = self.aggregator
        if self.agent.use_gpu and agg.backend != "nccl" and agg.native is None:
            return agg.host_all_gather(local)
        return agg.all_gather(local)

    def _validate(self, local, node):
        """Cross-check one native gather: every rank compares the node tensor RCCL
        produced with the control plane's host gather of the same blocks, bit for bit
        (NaN payloads included), and the ranks agree. All equal: counted in
        ``_ng.validated``. Any rank different: EVERY rank drops the native path from this
        refresh on (this refresh uses the host result) - no rank keeps gathering on a
        communicator its peers abandoned."""
        # the gather first, bounded: a D2H copy queued behind an ncclAllGather whose peer is
        # gone would block forever (_await_native aborts the communicator instead)
        self._await_native()
        ref = self.aggregator.host_all_gather(local)  # D2H of this rank's block
        got = node.detach().to("cpu")
        ok = tuple(got.shape) == tuple(ref.shape) and torch.equal(got.view(torch.int32), ref.view(torch.int32))
        if self.aggregator.min_over_ranks(1.0 if ok else 0.0) >= 1.0:
            self._ng.validated += 1
            return node
        import sys

        print(f"[rocmdash] rank {self.aggregator.rank}: native RCCL gather differs from the control-plane gather "
              f"(this rank {'matches' if ok else 'differs'}); every rank gathers through the host from now on",
              file=sys.stderr, flush=True)
        if self.agent.device.type == "cuda":  # the publication enqueued above has landed
            torch.cuda.current_stream(self.agent.device).synchronize()
        self.aggregator.disable_native("native gather failed validation")
        self._ng = None
        self.validate_gathers = 0
        self.gather_status = "host (native gather failed validation)"
        return ref

    def prevalidate(self) -> dict:
        """Collective: run the start-up validation gathers now (every rank calls it at
        the same point), so a timed loop never carries their host synchronisations.
        Returns ``gather_report()``."""
        while self._ng is not None and self._ng.validated < self.validate_gathers:
            self.latest_snapshot()
        return self.gather_report()

    def gather_report(self) -> dict:
        """How this pipeline gathers: {"status", "validated", "transport"} (bench JSON,
        /metrics)."""
        ng = self._ng
        tr = self.aggregator.native
        rep = {
            "status": self.gather_status,
            "validated": int(ng.validated) if ng is not None else 0,
            "validate_target": int(self.validate_gathers),
            "transport": tr.describe() if (ng is not None and tr is not None and hasattr(tr, "describe")) else None,
            "error": self.aggregator.native_error,
        }
        if ng is not None and tr is not None and hasattr(tr, "view"):
            # RCCL's own view of this rank's communicator and the transports it logged
            # per peer (rocmdash.parallel.rccl_log): the record's proof of N ranks / xGMI
            v = tr.view()
            rep["rccl_nranks"], rep["rccl_rank"], rep["rccl_device"] = v["nranks"], v["rank"], v["device"]
            d = tr.transport_detail() if hasattr(tr, "transport_detail") else None
            rep["transport_detail"] = None if d is None else {k: d[k] for k in ("kinds", "peers", "via", "lines")}
        return rep

    def _fill_side(self, buf: np.ndarray) -> np.ndarray:
        """This rank's side rows into ``buf`` [side, 8]: source health, per-XCD
        busy / clock, then the control row (stop vote, this rank's own footprint and
        gather state, schema.CONTROL_FIELDS)."""
        H = len(HEALTH_SOURCES)
        self.agent.health_rows(buf[:H])
        buf[H:H + XCD_ROWS] = self.agent.xcd()
        ctl = buf[H + XCD_ROWS]
        ctl[:] = np.nan
        ctl[CONTROL_INDEX["stop"]] = self.stop_vote
        if self.footprint is not None:
            if self.footprint._thread is None:  # sampled off the refresh path from now on
                self.footprint.start()
            self.footprint.fill(ctl)  # a copy of the background thread's newest sample
        ctl[CONTROL_INDEX["gather_validated"]] = self._ng.validated if self._ng is not None else -1.0
        src = buf[H + XCD_ROWS + 1]
        src[:] = np.nan
        c = self.agent.smi_source.counts()
        if "raw_path" in c:
            for k in ("raw_path", "calibration_attempts", "calibration_matched", "calibration_promotions",
                      "calibration_final"):
                src[SOURCE_INDEX["smi_" + k]] = c[k]
        return buf

    def _local_stats(self, ev=None):
        """This rank's block: the stats kernel's [S, 8] (+ the side rows), enqueued in
        stream order. With ``host_out`` it is rank 0's pinned host buffer itself.

        The side rows are filled on the host BEFORE the stats launch (their footprint
        part is a copy of a background sample: no I/O here), so no host work sits between
        the launch and the gather. ``ev`` (timed refreshes): HIP events recorded right
        before the launch (ev[0]), right after it (ev[1]) and after the side rows' H2D
        copy (ev[4])."""
        S = len(self.series)
        if self.host_out:
            if self.health:
                self._fill_side(self._host[0, S:].numpy())  # the host writes them in place
            if ev is not None:
                ev[0].record()
                t0 = time.perf_counter()
            self.agent.refresh(out=self._host[0, :S], signal=_HOST_SIGNAL if _DONE_FLAG else 0)
            if ev is not None:
                self.launch_host_s = time.perf_counter() - t0
                ev[1].record()
            return self._host[0]
        if not self.health:
            if ev is not None:
                ev[0].record()
                t0 = time.perf_counter()
            out = self.agent.refresh()
            if ev is not None:
                self.launch_host_s = time.perf_counter() - t0
                ev[1].record()
                ev[4].record()
            return out
        if not self.agent.use_gpu:  # CPU: the agent's output tensor + host rows
            side = torch.from_numpy(self._fill_side(self._side.numpy()))
            return torch.cat([self.agent.refresh(), side])
        if self._local is None:  # a pipeline built with host_out that no longer uses it
            self._local = torch.empty((self.rows, NUM_STATS), dtype=torch.float32, device=self.agent.device)
        local = self._local
        self._fill_side(self._side.numpy())
        if ev is not None:
            ev[0].record()
            t0 = time.perf_counter()
        self.agent.refresh(out=local[:S])
        if ev is not None:
            self.launch_host_s = time.perf_counter() - t0  # host time between the two events
            ev[1].record()
        local[S:].copy_(self._side, non_blocking=True)  # tiny H2D from pinned memory behind the kernel
        if ev is not None:
            ev[4].record()
        return local

    def _gather_timed(self):
        if not self.agent.use_gpu:  # CPU path: host clocks are the device clocks
            t0 = time.perf_counter()
            local = self._local_stats()
            t1 = time.perf_counter()
            node = self._native_gather(local) if self._ng is not None else self._fallback_gather(local)
            self._stage_host = (t1 - t0, time.perf_counter() - t1)
            return node
        if self._events is None:
            # [0] before the stats launch, [1] after it, [2] after the gather, [3] after
            # the publish kernel, [4] after the side rows' H2D copy
            self._events = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        ev = self._events
        if self.host_out:
            self._local_stats(ev)
            node = self._host
            self._timed = "host_out"
        else:
            local = self._local_stats(ev)
            if self._ng is not None:
                node = self._native_gather(local, ev)
                self._timed = "native" if self._ng is not None else "fallback"
            else:
                node = self._fallback_gather(local)
                ev[2].record()
                self._timed = "fallback"
        self._stage_host = None
        return node

    def stage_seconds(self) -> dict:
        """Device time of the last timed gather() (HIP events; host clocks on the CPU),
        in seconds: ``stats_kernel`` (the span between HIP events recorded right before
        and after the window-stats launch call: on an idle GPU the first event completes at
        once, so the span holds the host's launch call as well as the kernel),
        ``stats_launch_host`` (that launch call's host time: the kernel's own device time
        is about ``stats_kernel - stats_launch_host`` then), ``side_rows_h2d`` (the side rows' copy
        from pinned memory, service pipelines), ``allgather`` (the native
        ``ncclAllGather`` alone on the native path, including the wait for the slowest
        rank; the host gather on the fallback) and ``publish``. Empty when timing is off."""
        if not self.device_timing:
            return {}
        if self._stage_host is not None:
            return {"stats_kernel": self._stage_host[0], "allgather": self._stage_host[1]}
        if self._events is None:
            return {}
        ev = self._events
        kind = getattr(self, "_timed", "host_out")
        last = {"host_out": 1, "fallback": 2, "native": 3}[kind]
        ev[last].synchronize()  # elapsed_time needs both events complete
        out = {"stats_kernel": ev[0].elapsed_time(ev[1]) * 1e-3}
        if getattr(self, "launch_host_s", None) is not None:
            # the host's launch call between those two events: on an idle GPU the first
            # event completes at once and the span is mostly this (HIP's idle wake-up)
            out["stats_launch_host"] = self.launch_host_s
        if kind != "host_out":
            out["side_rows_h2d"] = ev[1].elapsed_time(ev[4]) * 1e-3
            out["allgather"] = ev[4].elapsed_time(ev[2]) * 1e-3
        if kind == "native":
            out["publish"] = ev[2].elapsed_time(ev[3]) * 1e-3
        return out

    def close(self) -> None:
        """Stop this pipeline's background footprint sampler (if it started one)."""
        if self.footprint is not None:
            self.footprint.stop()

    def _to_host(self, node) -> np.ndarray:
        """Rank 0: the node statistics [N, S, 8] on the host (synchronises the stream).
        With ``health`` the health rows are split off into ``last_health``."""
        if self._host is None:
            full = node.detach().cpu().numpy()
        else:
            if self._ng is not None and node is self._ng.out and self._ng.host is not None:
                self._await_native()  # the publish kernel's tagged words, copied into _host
                return self.split_health(self._host.numpy())
            if self.agent.device.type != "cuda":  # CPU stand-in of the native path, after a fallback
                self._host.copy_(node)
                return self.split_health(self._host.numpy())
            stream = torch.cuda.current_stream(self.agent.device)
            if not self.host_out:
                self._host.copy_(node, non_blocking=True)
                stream.synchronize()
            else:
                # host-out: the stats kernel's outputs carry their refresh's number (or its
                # last workgroup flags completion) in mapped host memory, ~10 us before the
                # stream's end-of-kernel signal. HIP events need the stream synchronised
                # (device_timing); tagged outputs reach the buffer through wait_refresh()
                # either way.
                if self.device_timing:
                    stream.synchronize()
                if not self.agent.wait_refresh():
                    stream.synchronize()
                    if self.agent.refresh_seq and not self.agent.wait_refresh(1.0):
                        raise RuntimeError("stats kernel outputs never carried the refresh's signal")
            full = self._host.numpy()
        return self.split_health(full)

    def split_health(self, full: np.ndarray) -> np.ndarray:
        """[N, rows, 8] -> the [N, S, 8] statistics; the side rows (if any) go to
        ``last_health`` / ``last_xcd`` / ``last_stop``."""
        if not self.health:
            return full
        S = len(self.series)
        H = len(HEALTH_SOURCES)
        self.last_health = full[:, S:S + H].copy()
        self.last_xcd = full[:, S + H:S + H + XCD_ROWS].copy()
        self.last_control = full[:, S + H + XCD_ROWS].copy()
        self.last_source = full[:, S + H + XCD_ROWS + 1].copy()
        self.last_stop = self.last_control[:, CONTROL_INDEX["stop"]].copy()
        return full[:, :S]

    def stop_votes(self) -> np.ndarray | None:
        """Every rank's stop vote carried by the last refresh's gather ([N]; None
        without side rows). Rank 0 has them on the host already; the other ranks copy
        the one column from the gathered tensor."""
        if not self.health:
            return None
        if self.is_root and self.last_stop is not None:
            return self.last_stop
        if self._node is None:
            return None
        S = len(self.series)
        col = self._node[:, S + len(HEALTH_SOURCES) + XCD_ROWS, CONTROL_INDEX["stop"]]
        return col.cpu().numpy() if hasattr(col, "cpu") else np.asarray(col)

    def _expand(self, node_host: np.ndarray):
        ids, infos = list(self.gpu_ids), self.infos
        if self.render_gpus > len(ids):
            reps = -(-self.render_gpus // len(ids))
            node_host = np.tile(node_host, (reps, 1, 1))[: self.render_gpus]
            infos = (infos * reps)[: self.render_gpus]
            ids = [str(i) for i in range(self.render_gpus)]
        return node_host, ids, infos

    def render_payload(self, node_host: np.ndarray):
        """Rank 0: the refresh's frame JSON from the gathered [N, S, 8] stats. The
        layout of a pipeline is fixed, so the native renderer is compiled once per
        selection (CompiledFrame) and each refresh renders straight from the array."""
        sel_key = None if self.selected is None else tuple(self.selected)
        if self._compiled is None or self._compiled_sel != sel_key:
            snap = self.snapshot(node_host)
            sel = self.selected if self.selected is not None else snap.gpu_ids
            try:
                self._compiled = CompiledFrame(snap, sel, use_gauge=self.use_gauge, extended=self.extended)
            except RuntimeError:  # no native renderer / a layout it does not escape
                self._compiled = False
            self._compiled_sel = sel_key
            if not self._compiled:
                return render_frame_json(snap, sel, use_gauge=self.use_gauge, extended=self.extended)
        if not self._compiled:
            snap = self.snapshot(node_host)
            sel = self.selected if self.selected is not None else snap.gpu_ids
            return render_frame_json(snap, sel, use_gauge=self.use_gauge, extended=self.extended)
        host, _, _ = self._expand(node_host)
        return self._compiled.render(host[:, :, LAST], host)

    def snapshot(self, node_host: np.ndarray) -> NodeSnapshot:
        node_host, ids, infos = self._expand(node_host)
        values = node_host[:, :, LAST]
        health = None
        if self.last_health is not None and len(self.last_health) == len(ids):
            health = SourceHealth(self.last_health, [(i["smi_backend"], i["counter_backend"]) for i in infos],
                                  self.agent.cfg.stale_periods)
        return NodeSnapshot(
            gpu_ids=ids,
            card_models=[i["card_model"] for i in infos],
            columns=self.series,
            values=values,
            power_limits=[i["power_limit_w"] for i in infos],
            product_names=[i["product_name"] for i in infos],
            window=node_host,
            window_series=self.series,
            source_health=health,
            xcd=self.last_xcd if self.last_xcd is not None and len(self.last_xcd) == len(ids) else None,
        )

    def sample_phase(self, sample: bool = True):
        """Step 1. Returns (t0, t1): when this refresh's sample started and when it was
        in the rings. With ``prefetch`` the sample was requested at the end of the
        previous sample phase, so t0 is that request's time."""
        t0 = time.perf_counter()
        if not sample:
            return t0, t0
        with trace_range("rocmdash.sample"):
            if self.sampling == "free":
                if self._free_calls is None:
                    self.start_sampling()
                self._free_calls, t0 = self.agent.wait_fresh(self._free_calls)
                return t0, time.perf_counter()
            if not self.prefetch:
                self.agent.sample()
                return t0, time.perf_counter()
            if self._prefetch_t0 is None:  # first refresh: nothing in flight yet
                self.agent.request_sample()
                self._prefetch_t0 = t0
            t0 = self._prefetch_t0
            self.agent.wait_sample()
            t1 = self._prefetch_t0 = time.perf_counter()
            self.agent.request_sample()
        return t0, t1

    def start_sampling(self) -> None:
        """Free-running sampling: start the agent's sources now (the bench does it before
        its warm-up; otherwise the first refresh does)."""
        if self.sampling != "free":
            raise ValueError("start_sampling() is for sampling='free'")
        if self._free_calls is None:
            self._free_calls = self.agent.start_free()

    def stop_sampling(self) -> None:
        """Stop free-running sampling (closed-loop reads work again afterwards)."""
        if self._free_calls is not None:
            self.agent.stop()
            self._free_calls = None

    def step(self, sample: bool = True, render: bool = True):
        """One refresh. Returns (payload_json or None, StepTiming).

        With ``prefetch`` the sample for the NEXT refresh is requested on the native
        sampler threads as soon as this refresh's sample is in, so it overlaps this
        refresh's statistics launch, all-gather and frame (none of which needs it).
        The reported latency still runs from the start of this refresh's own sample
        to its payload."""
        t0, t1 = self.sample_phase(sample)
        with trace_range("rocmdash.stats+allgather"):
            node = self.gather()
        payload = None
        if self.is_root:
            with trace_range("rocmdash.d2h"):
                host = self._to_host(node)
            t2 = time.perf_counter()
            if render:
                with trace_range("rocmdash.render"):
                    payload = self.render_payload(host)
        else:
            if self.agent.use_gpu or self._ng is not None:
                self._sync_gathered()
            t2 = time.perf_counter()
        t3 = time.perf_counter()
        timing = StepTiming(
            sample_ms=(t1 - t0) * 1e3,
            device_ms=(t2 - t1) * 1e3,
            render_ms=(t3 - t2) * 1e3,
            total_ms=(t3 - t0) * 1e3,
            payload_bytes=len(payload) if payload else 0,
        )
        return payload, timing

    def _sync_gathered(self) -> None:
        """A non-root rank: wait until this refresh's gather is done (flag, else the
        stream), so no rank runs ahead of the node's refresh."""
        if self._ng is not None:
            self._await_native()
            return
        if self.agent.device.type == "cuda":
            torch.cuda.current_stream(self.agent.device).synchronize()

    def _await_native(self) -> None:
        """Wait for the last native gather's publication, bounded
        (rocmdash.parallel.node.await_publication): past ``collective_timeout_s`` - or as
        soon as the communicator reports an error - the communicator is aborted and this
        raises, so the service exits for a restart (rocmdash.serve) and the bench fails
        loudly instead of hanging. A superseded publication fails at once."""
        from ..parallel.node import PublicationSuperseded, await_publication

        tr = self.aggregator.native
        try:
            await_publication(self._ng.pub, self._ng.seq, tr, self.collective_timeout_s, abandon=self.aggregator.abandon)
        except PublicationSuperseded:
            raise
        except RuntimeError:
            self.aggregator.native = None
            self._ng = None
            raise

    def latest_snapshot(self) -> NodeSnapshot | None:
        """Gather + snapshot without rendering (the in-process data source of the app)."""
        node = self.gather()
        self._node = node
        if not self.is_root:
            if self._ng is not None and node is self._ng.out:
                self._await_native()  # bounded: stop_votes() then reads the gathered tensor
            return None
        host = self._to_host(node).copy()
        return self.snapshot(host)


class PipelinedRefresher:
    """Refresh loop with rank 0's rendering overlapped with the next refresh.

    Rank 0 hands refresh i's node tensor to a render thread and immediately goes on
    with refresh i+1 (its sample - prefetched on the native sampler threads when the
    pipeline prefetches -, stats launch and all-gather). The native renderer releases
    the GIL, so the refresh *rate* is bounded by max(sample, gather, render) instead of
    sample-wait + gather + render: this is what keeps rank 0's 4 + 4N figures off the
    critical path of the whole node at N = 8. Each refresh's latency (sample start ->
    payload ready) is recorded unchanged. At most one render is outstanding and the
    D2H buffers are double-buffered, so nothing is skipped or reused early.
    """

    def __init__(self, pipe: NodePipeline):
        from concurrent.futures import ThreadPoolExecutor

        if pipe.host_out:  # the render thread reads double buffers filled by D2H copies
            raise ValueError("PipelinedRefresher needs a NodePipeline built with allow_host_out=False")
        self.pipe = pipe
        if pipe._ng is not None:
            pipe._ng.host = None  # rank 0 copies into its own double buffers: publish the signal only
        self.is_root = pipe.is_root
        self._pool = ThreadPoolExecutor(1, thread_name_prefix="rocmdash-render") if self.is_root else None
        self._pending = None
        self._i = 0
        self._bufs = None
        if self.is_root and pipe.agent.use_gpu:
            shape = (pipe.aggregator.world_size, pipe.rows, NUM_STATS)
            self._bufs = [torch.empty(shape, dtype=torch.float32, pin_memory=True) for _ in range(2)]
        self.latencies_ms: list = []
        self.parts_ms: list = []  # (sample, device+gather+d2h) per refresh
        self.payload_bytes = 0
        self.last_payload = None

    def _render(self, host: np.ndarray, t0: float) -> None:
        p = self.pipe
        with trace_range("rocmdash.render"):
            payload = p.render_payload(host)
        self.latencies_ms.append((time.perf_counter() - t0) * 1e3)
        self.payload_bytes = len(payload)
        self.last_payload = payload

    def step(self) -> None:
        p = self.pipe
        t0, t1 = p.sample_phase()
        with trace_range("rocmdash.stats+allgather"):
            node = p.gather()
        if p._ng is not None and node is p._ng.out:
            p._await_native()  # bounded: a stream synchronisation behind a lost peer never returns
        if self.is_root:
            with trace_range("rocmdash.d2h"):
                if self._bufs is not None:
                    buf = self._bufs[self._i & 1]
                    buf.copy_(node, non_blocking=True)
                    torch.cuda.current_stream(p.agent.device).synchronize()
                    host = p.split_health(buf.numpy())
                else:
                    host = p.split_health(node.detach().cpu().numpy().copy())
            t2 = time.perf_counter()
            if self._pending is not None:
                self._pending.result()  # at most one render in flight (buffer i-1 in use)
            self._pending = self._pool.submit(self._render, host, t0)
        else:
            if p.agent.use_gpu:
                torch.cuda.current_stream(p.agent.device).synchronize()
            t2 = time.perf_counter()
        self.parts_ms.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3))
        self._i += 1

    def flush(self) -> None:
        if self._pending is not None:
            self._pending.result()
            self._pending = None

    def close(self) -> None:
        self.flush()
        if self._pool is not None:
            self._pool.shutdown(wait=True)
