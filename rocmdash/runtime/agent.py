"""Per-GPU telemetry agent: sources -> pinned rings -> device windows -> stats tensor.

One agent per rank (one process per GPU). It owns
  * an amd-smi source (10 Hz default) and a rocprofiler-sdk device-counting source
    (100 Hz default) for ITS GPU, or synthetic sources of the same layout;
  * one pinned-host ``SeriesRing`` per source and a native ``Sampler`` that fills it,
    either on a background thread at a fixed rate or closed-loop (``sample()``);
  * a ``DeviceWindowSet`` that keeps every series' sorted window resident on the GPU
    and launches the window-stats kernel over every series in ONE launch, writing a
    ``[S, 8]`` float32 tensor; the kernel pulls the entering rows straight from the
    mapped pinned ring (a ``hipMemcpyAsync`` staging copy only before a full re-sort).

Reference counterpart: none on the device side. The reference's data source is the
external exporter behind Prometheus (``app.py:167-178``); the series and labels it
reads are the first five SMI columns here (``rocmdash.models.schema``).
"""

from __future__ import annotations

import os
import time
from dataclasses import dataclass

import numpy as np

from ..config import SamplerConfig
from ..models.gpu_models import normalize_power_limit_w
from ..models.schema import (
    CTR_FIELDS,
    HEALTH_INDEX,
    HEALTH_SOURCES,
    HEALTH_SPLIT,
    NUM_STATS,
    SMI_FIELDS,
    SMI_LIVE_FIELDS,
    SMI_TABLE_FIELDS,
    XCDS,
)
from ..ops.window_stats import DEFAULT_PCT, window_stats_reference
from . import native as _nat


def _current_raw_stream(device_index: int) -> int:
    """The caller's current HIP stream on ``device_index`` as a raw handle - what
    ``torch.cuda.current_stream(d).cuda_stream`` returns, without building the Stream
    object (~1.3 us per refresh on the box, tools/probes/probe_refresh_flag.py)."""
    import torch

    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if raw is not None:
        return int(raw(device_index))
    return torch.cuda.current_stream(device_index).cuda_stream


@dataclass
class AgentInfo:
    gpu_id: str
    device_index: int
    bdf: int
    card_model: str
    product_name: str
    power_limit_w: float | None
    smi_backend: str
    counter_backend: str
    series: tuple

    def as_dict(self) -> dict:
        return dict(self.__dict__)


class GpuAgent:
    """Telemetry for one GPU. ``device`` is a torch device (cuda:i, or cpu for the
    CPU reference path used by tests and CPU-only dashboards)."""

    def __init__(
        self,
        device_index: int = 0,
        *,
        source: str = "auto",  # "auto" | "hw" | "synthetic" | "replay"
        # "auto" | "hw" | "synthetic" | "off" | "node": this GPU's rows from the node's
        # counter process (rocmdash.runtime.counterd) through shared memory - no counting
        # context, no busy-polling runtime thread in this process
        counters: str = "auto",
        cfg: SamplerConfig | None = None,
        seed: int | None = None,
        use_gpu: bool | None = None,
        pct=DEFAULT_PCT,
        replay=None,  # source="replay": a recording (path or dict, rocmdash.runtime.record)
    ):
        import torch

        self.cfg = cfg or SamplerConfig()
        self.pct = tuple(float(p) for p in pct)
        self.nat = _nat.load()
        nat = self.nat
        if use_gpu is None:
            use_gpu = torch.cuda.is_available()
        self.use_gpu = bool(use_gpu)
        self.device = torch.device("cuda", device_index) if self.use_gpu else torch.device("cpu")
        self.device_index = device_index
        seed = (0x5EED + 7919 * device_index) if seed is None else seed

        # ---- identify the GPU (bdf) so amd-smi and rocprofiler talk about the same one
        bdf = 0
        if self.use_gpu:
            bdf = int(nat.hip_device_bdf(device_index))
            # the runtime is up now (its counter-read state is fixed): undo the init
            # pin so later threads (samplers pin themselves; RCCL, torch, HTTP) get
            # the process's full CPU mask again
            from .placement import restore_affinity

            restore_affinity()
        self.bdf = bdf

        # ---- sources
        want_hw = source in ("auto", "hw")
        smi = None
        ctr = None
        replayed = None
        if source == "replay":
            from .record import load_recording

            rec = load_recording(replay) if isinstance(replay, str) else replay
            if rec is None or "smi_rows" not in rec:
                raise ValueError("source='replay' needs replay=<recording path or dict> with smi rows")
            info = {k: v for k, v in dict(rec.get("info", {})).items() if v is not None}
            info.setdefault("model_number", info.get("card_model", ""))
            info = {k: info[k] for k in ("model_number", "product_name", "power_limit_w", "vram_total_mb") if k in info}
            smi = nat.make_replay_source("smi", rec["smi_rows"], info)
            if "counter_rows" in rec and counters != "off":
                ctr = nat.make_replay_source("counter", rec["counter_rows"], {})
            replayed = True
        elif want_hw and nat.amdsmi_gpu_count() > 0:
            try:
                smi = nat.make_smi_source(bdf, device_index)
            except RuntimeError:
                if source == "hw":
                    raise
        elif source == "hw":
            raise RuntimeError("source='hw' but amd-smi found no GPU")
        if smi is None:
            smi = nat.make_synthetic_source("smi", seed)

        if replayed:
            pass  # counters come from the recording (or none)
        elif counters == "node":
            from .counterd import ring_path

            shm = os.environ.get("ROCMDASH_COUNTER_SHM", "")
            if not shm:
                raise RuntimeError("counters='node' needs ROCMDASH_COUNTER_SHM (the node counter process's directory)")
            ctr = nat.make_shm_source(ring_path(shm, device_index), float(self.cfg.counter_hz))
        elif counters in ("auto", "hw"):
            if _nat.counters_ready():
                try:
                    # the whole physical GPU: every compute partition's agent when the
                    # GPU is partitioned (topology.node_plan), the one agent otherwise
                    ctr = nat.make_counter_source_all(bdf, device_index)
                except RuntimeError:
                    if counters == "hw":
                        raise
            elif counters == "hw":
                raise RuntimeError(f"counters='hw' but device counting is unavailable: {_nat.counters_status()}")
            if ctr is None and smi.backend == "synthetic":
                ctr = nat.make_synthetic_source("counter", seed)
            elif ctr is None and _nat.counters_requested():
                # counters were requested for this process but this GPU's could not be
                # configured: keep the series layout every rank shares, with NaN rows
                ctr = nat.make_null_source("counter")
        elif counters == "synthetic":
            ctr = nat.make_synthetic_source("counter", seed)
        self.smi_source = smi
        self.ctr_source = ctr
        self._requested = False
        self._checked_out = None
        self._seq = 0

        # ---- rings + samplers (pinned host memory when a GPU consumes them)
        nat.set_pinned_host_rings(self.use_gpu)
        self.smi_ring = nat.SeriesRing(len(SMI_FIELDS), self.cfg.ring_capacity)
        self.smi_sampler = nat.Sampler(smi, self.smi_ring, self.cfg.smi_hz)
        self.rings = [self.smi_ring]
        self.samplers = [self.smi_sampler]
        self.series = tuple(SMI_FIELDS)
        if ctr is not None:
            self.ctr_ring = nat.SeriesRing(len(CTR_FIELDS), self.cfg.ring_capacity)
            self.ctr_sampler = nat.Sampler(ctr, self.ctr_ring, self.cfg.counter_hz)
            self.rings.append(self.ctr_ring)
            self.samplers.append(self.ctr_sampler)
            self.series = self.series + tuple(CTR_FIELDS)
        else:
            self.ctr_ring = None
            self.ctr_sampler = None

        self.sampler_cpus = []
        if self.cfg.pin_samplers == "numa" and bdf:
            self.sampler_cpus = numa_local_cpus(bdf)
        elif self.cfg.pin_samplers == "init" and bdf:  # the node the runtime started on (placement.py)
            self.sampler_cpus = init_node_cpus()
        for smp in self.samplers:
            smp.set_spin_us(float(self.cfg.spin_us))
            if self.sampler_cpus:
                smp.set_affinity(self.sampler_cpus)

        # ---- device mirror + output
        self.window = self.cfg.window
        self.dws = None
        if self.use_gpu:
            if self.cfg.long_window:  # HBM-resident window, multi-workgroup radix select
                self.dws = nat.LongWindowSet(self.window, device_index)
            else:
                self.dws = nat.DeviceWindowSet(self.window, device_index)
            self._signals = isinstance(self.dws, nat.DeviceWindowSet)  # refresh(signal=...) supported
            for r in self.rings:
                self.dws.add_ring(r)
            self.out = torch.empty((len(self.series), NUM_STATS), dtype=torch.float32, device=self.device)
        else:
            self.out = torch.empty((len(self.series), NUM_STATS), dtype=torch.float32)

        inf = smi.info()
        card_model = inf.get("model_number") or "unknown"
        self.info = AgentInfo(
            gpu_id=str(inf.get("index", -1) if inf.get("index", -1) >= 0 else device_index),
            device_index=device_index,
            bdf=bdf,
            card_model=card_model,
            product_name=inf.get("product_name") or "",
            power_limit_w=normalize_power_limit_w(inf.get("power_limit_w")) if inf.get("power_limit_w") else None,
            smi_backend=smi.backend,
            counter_backend=ctr.backend if ctr is not None else "off",
            series=self.series,
        )

    # ------------------------------------------------------------------ sampling
    def sample(self) -> int:
        """Closed-loop: take one sample from every source now (caller's thread).
        Returns the number of rows pushed."""
        others = self.samplers[1:]
        for s in others:  # device counters on their worker thread, concurrently
            s.request()
        n = int(bool(self.samplers[0].sample_once()))
        for s in others:
            n += int(bool(s.wait()))
        return n

    def request_sample(self) -> None:
        """Start one sample of every source on the samplers' native worker threads and
        return at once (no GIL held while they read): the next refresh's sample runs
        while this refresh's statistics, gather and frame are produced."""
        if self._requested:
            raise RuntimeError("a sample request is already pending")
        for s in self.samplers:
            s.request()
        self._requested = True

    def wait_sample(self) -> int:
        """Wait for the pending request_sample(); returns the number of rows pushed."""
        if not self._requested:
            return 0
        n = 0
        for s in self.samplers:
            n += int(bool(s.wait()))
        self._requested = False
        return n

    def start(self) -> None:
        """Background sampling at the configured rates (native threads). A source fed by
        the node's counter process runs free instead: each call hands over the next row
        that process published (sleeping until it is due), so none is lost or repeated
        whatever the two clocks do."""
        for s in self.samplers:
            if s.source.backend == "node-counterd":
                s.start_free(4.0 * s.hz)
            else:
                s.start()

    def start_free(self) -> list:
        """Free-running sampling: every source reads back to back on its own native
        thread, unpaced, and refreshes take whatever rows arrived (``wait_fresh``). The
        bench's N > 1 mode: no rank's read waits for the node's refresh, so the node does
        not refresh at the pace of its slowest rank's read tail. Returns the sources'
        completed-call counts at the start (the first ``wait_fresh`` baseline)."""
        self.wait_sample()  # no closed-loop request may be left pending (SPSC ring)
        calls = [int(s.calls()) for s in self.samplers]
        max_hz = float(os.environ.get("ROCMDASH_FREE_MAX_HZ", "50000"))
        for s in self.samplers:
            s.start_free(max_hz)
        return calls

    def wait_fresh(self, after: list, timeout_s: float = 1.0) -> tuple:
        """Free-running: wait (spinning, GIL released) until every source has completed
        a read after the counts ``after``, at most ``timeout_s`` per source (a stuck
        source shows up as stale in the health rows, it does not stall the node).
        Returns (counts now, perf_counter seconds at which the OLDEST of the sources'
        newest reads started - the start of this refresh's sample)."""
        now = [int(s.wait_calls(int(c) + 1, timeout_s)) for s, c in zip(self.samplers, after)]
        t0 = min(s.last_start_ns() for s in self.samplers) * 1e-9
        return now, t0

    def stop(self) -> None:
        for s in self.samplers:
            s.stop()

    def prefill(self, rows: int | None = None) -> None:
        """Fill every ring with ``rows`` samples (default: one window) closed-loop, so a
        window is full before the first refresh (benchmarks, demos)."""
        rows = self.window if rows is None else rows
        for _ in range(rows):
            self.sample()

    def prefill_bulk(self, rows: int, seed: int = 0, like: str = "normal") -> int:
        """Fill every ring's window with ``rows`` generated rows, staged to the device
        window ring-full by ring-full so none is lost. For kernel-cost measurements of
        windows far longer than the live sources can fill in a run (2^24 samples = 23 min
        of counter reads at 12 kHz): callers label it. ``like``:

        * ``"normal"`` - telemetry-like numbers (integer readings in a band for half the
          columns, continuous N(50, 10) for the others);
        * ``"live"`` - rows drawn (whole rows, with replacement) from the rows the live
          sources already put in each ring: the window then holds the node's own
          telemetry distribution, so the rows that keep arriving do not drift every
          percentile away from the generated bulk (the node window's
          bracket misses over a "normal" bulk were that drift, not the data's).

        Returns the rows pushed per ring."""
        import torch

        rng = np.random.default_rng(seed + 7919 * self.device_index)
        pools = None
        if like == "live":
            pools = []
            for r in self.rings:
                have, _ = r.window(min(int(self.cfg.ring_capacity), 1 << 16))
                have = np.asarray(have, dtype=np.float32)
                if not len(have):
                    raise RuntimeError("prefill_bulk(like='live'): no live rows in the rings yet")
                pools.append(have)
        elif like != "normal":
            raise ValueError(f"prefill_bulk: like={like!r}")
        block = min(rows, max(1, self.cfg.ring_capacity // 2))
        t = time.time_ns()
        done = 0
        while done < rows:
            k = min(block, rows - done)
            for i, r in enumerate(self.rings):
                if pools is not None:
                    x = pools[i][rng.integers(0, len(pools[i]), k)]
                else:
                    x = rng.normal(50.0, 10.0, (k, r.width)).astype(np.float32)
                    x[:, ::2] = np.rint(x[:, ::2])  # half the columns integer-valued
                r.push_many(x, np.arange(t, t + k, dtype=np.uint64))
            t += k
            done += k
            if self.dws is not None:
                self.refresh()  # stage these rows into the device window
                torch.cuda.synchronize(self.device)
        return done

    def xcd(self) -> np.ndarray:
        """[2, 8] float32: per-XCD busy (%) and gfx clock (MHz) from the latest SMU
        sample (csrc/sources.cpp; NaN where the source has none, e.g. replay)."""
        out = np.full((2, XCDS), np.nan, dtype=np.float32)
        d = self.smi_source.xcd_detail()
        if d is not None:
            n = min(XCDS, len(d["busy"]))
            out[0, :n] = d["busy"][:n]
            out[1, :n] = d["clock_mhz"][:n]
        return out

    def info_calibration(self) -> str:
        """The amd-smi source's current raw-table calibration text ("" for other sources):
        it changes when a retry runs (csrc/sources.h RawCalibrationPolicy)."""
        return str(self.smi_source.info().get("metrics_calibration") or "")

    def sampler_stats(self) -> list:
        return [s.stats() for s in self.samplers]

    def health_rows(self, out: np.ndarray, now_ns: int | None = None) -> np.ndarray:
        """Fill ``out`` [len(HEALTH_SOURCES), 8] float32 with each source's health
        (schema.HEALTH_FIELDS): exact sample / failure counts, overruns, age of the
        newest row in seconds (NaN: none yet), the source's rate and 1 if present.
        This rank's block of the per-rank health the node tensor carries to rank 0."""
        now_ns = time.time_ns() if now_ns is None else now_ns
        out.fill(np.nan)
        by_kind = {s.source.kind: (s, r) for s, r in zip(self.samplers, self.rings)}
        H = HEALTH_INDEX
        for i, kind in enumerate(HEALTH_SOURCES):
            if kind not in by_kind:
                out[i, H["present"]] = 0.0
                continue
            smp, ring = by_kind[kind]
            n_ok, n_fail, n_over = smp.counts()
            out[i, H["samples_hi"]], out[i, H["samples_lo"]] = divmod(n_ok, HEALTH_SPLIT)
            out[i, H["failures_hi"]], out[i, H["failures_lo"]] = divmod(n_fail, HEALTH_SPLIT)
            out[i, H["overruns"]] = n_over
            last = ring.last_timestamp
            out[i, H["age_s"]] = (now_ns - last) * 1e-9 if last else np.nan
            out[i, H["hz"]] = smp.hz
            out[i, H["present"]] = 1.0
        return out

    def sample_counts(self) -> dict:
        """Cumulative counts for fresh-sample accounting (bench.py): rows pushed per
        source and the SMU table publications seen by the amd-smi source."""
        out = {}
        for s in self.samplers:
            if s.source.backend != "unavailable":  # a null source pushes NaN rows
                out[s.source.kind + "_rows"] = int(s.counts()[0])
        c = self.smi_source.counts()
        if "raw_table_changes" in c and c.get("raw_reads", 0) > 0:
            out["smi_table_changes"] = int(c["raw_table_changes"])
        return out

    def fresh_breakdown(self, before: dict, after: dict) -> dict:
        """``fresh_samples`` split by where the values came from: device counters, the
        live used-VRAM column, the SMU-table series."""
        d = {k: after.get(k, 0) - before.get(k, 0) for k in after}
        smi_rows = d.get("smi_rows", 0)
        return {"counters": int(d.get("counter_rows", 0) * len(CTR_FIELDS)),
                "used_vram": int(smi_rows * len(SMI_LIVE_FIELDS)),
                "smu_table": int(min(d.get("smi_table_changes", smi_rows), smi_rows) * len(SMI_TABLE_FIELDS))}

    def fresh_samples(self, before: dict, after: dict) -> int:
        """Series values that carried new data between two ``sample_counts()``:
        every counter row (cumulative hardware counters, each row a new delta) times
        its series; every amd-smi row's live column (used VRAM); the SMU-table
        columns once per table the firmware published (``raw_table_changes``), or
        per row when the source cannot tell (amd-smi library decoding, synthetic and
        replayed sources, whose every row is new). Total VRAM is a constant and never
        counts."""
        d = {k: after.get(k, 0) - before.get(k, 0) for k in after}
        n = d.get("counter_rows", 0) * len(CTR_FIELDS)
        smi_rows = d.get("smi_rows", 0)
        n += smi_rows * len(SMI_LIVE_FIELDS)
        table = d.get("smi_table_changes", smi_rows)
        n += min(table, smi_rows) * len(SMI_TABLE_FIELDS)
        return int(n)

    # ------------------------------------------------------------------ refresh
    def refresh(self, out=None, signal: int = 0):
        """Enqueue the stats kernel (+ staging copies before a full re-sort); returns the [S, 8] tensor
        (device tensor on GPU: valid in stream order, no host sync here). ``out``: write
        the statistics there instead - any device-accessible float32 [S, 8] buffer, e.g.
        pinned host memory that the kernel then fills directly (no D2H copy).
        ``signal`` (GPU): how ``wait_refresh()`` learns the outputs are in - 0 none
        (synchronise the stream; no epilogue in the kernel), 1 completion flag, 2 tagged
        outputs (``out`` is pinned host memory; ``wait_refresh()`` fills it from the
        kernel's {value, refresh} words - csrc/device_window.h)."""
        if self.dws is not None:
            dst = self.out if out is None else out
            if dst is not self._checked_out:  # validated once per buffer (a refresh is ~3 us of native work)
                import torch

                if tuple(dst.shape) != tuple(self.out.shape) or dst.dtype != torch.float32 or not dst.is_contiguous():
                    raise ValueError(f"out must be a contiguous float32 {tuple(self.out.shape)} tensor")
                self._checked_out = dst
            stream = _current_raw_stream(self.device_index)
            if self._signals:
                self._seq = self.dws.refresh(dst.data_ptr(), stream, *self.pct, signal)
            else:  # long windows: stream order only
                self.dws.refresh(dst.data_ptr(), stream, *self.pct)
                self._seq = 0
            return dst
        st = self._refresh_cpu()
        if out is not None:
            out.copy_(st)
            return out
        return st

    @property
    def refresh_seq(self) -> int:
        """Completion sequence number of the last ``refresh()`` (0: no signal)."""
        return int(self._seq or 0)

    def wait_refresh(self, timeout_s: float = 1.0) -> bool:
        """Spin until the last ``refresh()``'s kernels have written their outputs (its
        ``signal``: the completion flag in mapped host memory, or every tagged output
        word carrying the refresh's number - then copied to ``out``), seen before the
        stream's completion signal would be (csrc/device_window.cpp). False without a
        signal (CPU, unpinned rings, ``signal=0``) or on timeout: then synchronise the
        stream instead. The rest of the stream is NOT waited for."""
        if self.dws is None or not self._seq:
            return False
        return bool(self.dws.wait_done(self._seq, timeout_s))

    def _refresh_cpu(self):
        import torch

        blocks = []
        for r in self.rings:
            rows, _ = r.window(self.window)
            x = rows.T if len(rows) else np.full((r.width, 1), np.nan, dtype=np.float32)
            st = window_stats_reference(x, self.pct)
            if not len(rows):
                st[:, 6] = np.nan
                st[:, 7] = 0
            blocks.append(st)
        self.out.copy_(torch.from_numpy(np.concatenate(blocks, axis=0).astype(np.float32)))
        return self.out

    def export_window(self):
        """Every series' current window, sorted, as ``[S, 1 + W]`` float32 (element 0 =
        the number of valid samples, then the samples ascending, +inf after them): this
        rank's block of the node-wide window statistics (``rocmdash.parallel.node_window``).
        On a GPU the block is exported from the resident sorted windows the last
        ``refresh()`` left on the device (csrc/node_window.hip), in stream order."""
        import torch

        W = self.window
        if self.dws is not None:
            if not hasattr(self.dws, "export_sorted"):  # long windows never leave their GPU
                raise ValueError("a window of > 32768 samples is not exported: NodeWindowStats computes the node "
                                 "statistics of long windows by a distributed radix select (LongWindowSet.refresh_node)")
            buf = getattr(self, "_export", None)
            if buf is None:
                buf = self._export = torch.empty((len(self.series), W + 1), dtype=torch.float32, device=self.device)
            self.dws.export_sorted(buf.data_ptr(), torch.cuda.current_stream(self.device).cuda_stream)
            return buf
        out = np.full((len(self.series), W + 1), np.inf, dtype=np.float32)
        s = 0
        for r in self.rings:
            rows, _ = r.window(W)
            for c in range(r.width):
                v = np.sort(rows[:, c][~np.isnan(rows[:, c])]) if len(rows) else np.zeros(0, np.float32)
                out[s, 0] = len(v)
                out[s, 1 : 1 + len(v)] = v
                s += 1
        return torch.from_numpy(out)

    def window_host(self, ring_index: int = 0):
        """Newest window of a ring on the host (oldest first) - for tests/debug."""
        return self.rings[ring_index].window(self.window)

    def close(self) -> None:
        self.wait_sample()
        self.stop()
        self.dws = None


def now_ns() -> int:
    return time.time_ns()


def bdf_path(bdf: int) -> str:
    """amd-smi bdf id (domain<<32 | bus<<8 | dev<<3 | fn) -> sysfs PCI device dir."""
    return "/sys/bus/pci/devices/%04x:%02x:%02x.%x" % (bdf >> 32, (bdf >> 8) & 0xFF, (bdf >> 3) & 0x1F, bdf & 0x7)


def parse_cpulist(text: str) -> list:
    cpus = []
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.extend(range(int(lo), int(hi or lo) + 1))
    return cpus


def init_node_cpus() -> list:
    """CPUs of the NUMA node the placement calibration started the runtime on ([] if
    none was chosen) - where the runtime's own threads, its busy-polling async-events
    thread among them (threads.py), live."""
    from .placement import choice, numa_nodes

    c = choice() or {}
    node = c.get("node")
    return list(numa_nodes().get(int(node), [])) if node is not None else []


def numa_local_cpus(bdf: int) -> list:
    """CPUs on the GPU's NUMA node that this process may run on ([] if unknown). The
    sampler's sysfs reads and the driver's SMU / counter round trips then stay on the
    socket the GPU hangs off."""
    try:
        with open(bdf_path(bdf) + "/local_cpulist") as f:
            local = parse_cpulist(f.read())
        from .placement import process_cpus

        allowed = process_cpus()  # the process's CPUs, not the init pin (placement.py)
    except (OSError, ValueError, AttributeError):
        return []
    cpus = [c for c in local if c in allowed]
    return cpus if len(cpus) < len(allowed) else []  # all of them: nothing to pin
