"""Node exporter: ``/metrics`` with the ``amd_gpu_*`` series the dashboard queries.

Reference counterpart: the AMD device-metrics exporter the reference assumes is
scraped by Prometheus (``app.py:168-171``; not part of the reference repo). This
exporter is fed by rocmdash's own native pipeline:

  * ``LocalNodeSource``: one process samples every GPU of the node (a DaemonSet pod):
    one ``GpuAgent`` per device with background native samplers (amd-smi 10 Hz,
    device counters 100 Hz); a scrape refreshes every agent's device window (one
    window-stats launch per GPU) and renders latest values + window statistics;
  * ``PipelineSource``: rank 0 of the rank-per-GPU pipeline (``rocmdash.serve``)
    renders the RCCL-gathered node snapshot;
  * ``SyntheticSource``: a synthetic node (CPU tests, demos).

Every scrape also reports the exporter's own health: sampler counts/failures/
overruns, last sample age (staleness), scrape and refresh durations.

    python -m rocmdash.prom.exporter --port 9400            # all local GPUs
    python -m rocmdash.prom.exporter --synthetic 8 --port 9400
"""

from __future__ import annotations

import argparse
import logging
import socket
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy as np

from ..models.schema import STAT_INDEX
from ..utils.timing import LatencyHistogram
from ..viz.panels import NodeSnapshot
from .exposition import Exposition, render_snapshot

log = logging.getLogger("rocmdash.prom.exporter")
CONTENT_TYPE = "text/plain; version=0.0.4; charset=utf-8"
LAST = STAT_INDEX["last"]


class SnapshotSource:
    """Produces (NodeSnapshot, self_metrics: Exposition) per scrape."""

    def collect(self):  # pragma: no cover - interface
        raise NotImplementedError

    def close(self) -> None:
        pass


class SyntheticSource(SnapshotSource):
    def __init__(self, n_gpus: int = 8, seed: int = 0):
        from .mock import SyntheticNode

        self.node = SyntheticNode(n_gpus, seed=seed)

    def collect(self):
        self.node.step()
        cols = None
        rows = []
        for g in range(len(self.node.gpu_ids)):
            v = self.node.values(g)
            cols = tuple(v)
            rows.append([v[c] for c in cols])
        snap = NodeSnapshot(
            gpu_ids=list(self.node.gpu_ids),
            card_models=[self.node.card_model] * len(rows),
            columns=cols,
            values=rows,
        )
        return snap, None


class LocalNodeSource(SnapshotSource):
    """Every visible GPU in this process, background sampling, stats per scrape."""

    def __init__(self, devices=None, source: str = "auto", counters: str = "auto", cfg=None,
                 node_window: bool = False):
        from ..runtime import native

        native.load()
        if counters in ("auto", "hw"):
            native.enable_counters()
        import torch

        from ..runtime.agent import GpuAgent

        n = torch.cuda.device_count() if torch.cuda.is_available() else 0
        devices = list(range(n)) if devices is None else list(devices)
        if not devices:
            raise RuntimeError("no GPU visible to the exporter (use --synthetic N for a synthetic node)")
        self.agents = [GpuAgent(d, source=source, counters=counters, cfg=cfg) for d in devices]
        series = {a.series for a in self.agents}
        if len(series) != 1:
            raise RuntimeError(f"GPUs disagree on the series layout: {series}")
        self.series = self.agents[0].series
        for a in self.agents:
            a.start()
        self._lock = threading.Lock()
        self.last_refresh_s = 0.0
        self.refresh_hist = LatencyHistogram("rocmdash_refresh_latency_seconds", "Device refresh latency per scrape")
        self.node_window = bool(node_window)

    def collect(self):
        import torch

        with self._lock:
            t0 = time.perf_counter()
            outs = [a.refresh() for a in self.agents]  # one launch per GPU, all async
            host = np.stack([o.to("cpu", non_blocking=False).numpy() for o in outs])
            node_stats = self._node_window() if self.node_window else None
            self.last_refresh_s = time.perf_counter() - t0
            self.refresh_hist.observe(self.last_refresh_s)
        ids = [a.info.gpu_id for a in self.agents]
        if len(set(ids)) != len(ids):
            ids = [str(a.device_index) for a in self.agents]
        snap = NodeSnapshot(
            gpu_ids=ids,
            card_models=[a.info.card_model for a in self.agents],
            columns=self.series,
            values=host[:, :, LAST],
            power_limits=[a.info.power_limit_w for a in self.agents],
            product_names=[a.info.product_name for a in self.agents],
            window=host,
            window_series=self.series,
            node_window=node_stats,
            xcd=np.stack([a.xcd() for a in self.agents]),
        )
        exp = Exposition()
        now_ns = time.time_ns()
        for a, gid in zip(self.agents, ids):
            for sampler, ring in zip(a.samplers, a.rings):
                kind = sampler.source.kind
                backend = sampler.source.backend
                lab = {"gpu_id": gid, "source": kind, "backend": backend}
                st = sampler.stats()
                exp.add("rocmdash_sampler_samples_total", st["samples"], lab, "Rows pushed into the ring", "counter")
                exp.add("rocmdash_sampler_failures_total", st["failures"], lab, "Failed source reads", "counter")
                exp.add("rocmdash_sampler_overruns_total", st["overruns"], lab, "Missed sampling deadlines", "counter")
                exp.add("rocmdash_sampler_read_seconds", st["mean_us"] * 1e-6, lab, "Mean duration of one source read")
                last = ring.last_timestamp
                age = (now_ns - last) * 1e-9 if last else float("nan")
                exp.add("rocmdash_sample_age_seconds", age, lab, "Age of the newest sample (staleness)")
                # stale: no sample for `stale_periods` sampling periods (or never)
                limit = a.cfg.stale_periods / sampler.hz
                stale = 1.0 if (not last or age > limit) else 0.0
                exp.add("rocmdash_source_stale", stale, lab, "1 if the source produced no sample within stale_periods periods")
        exp.add("rocmdash_refresh_seconds", self.last_refresh_s, {}, "Device refresh (stats kernel + D2H) of the last scrape")
        self.refresh_hist.add_to(exp)
        torch.cuda.synchronize()
        return snap, exp

    def _node_window(self):
        """[S, 8] statistics over every local GPU's window: the sorted windows of all
        GPUs gathered on the first one (peer copies), one rank-selection launch."""
        import torch

        from ..parallel.node_window import node_window_reference

        blocks = [a.export_window() for a in self.agents]
        first = self.agents[0]
        if not blocks[0].is_cuda:
            return node_window_reference(np.stack([b.numpy() for b in blocks]), first.pct)
        node = torch.stack([b.to(first.device) for b in blocks]).contiguous()
        N, S, Wp1 = node.shape
        out = torch.empty((S, 8), dtype=torch.float32, device=first.device)
        first.nat.node_select(node.data_ptr(), N, S, Wp1 - 1, out.data_ptr(),
                              torch.cuda.current_stream(first.device).cuda_stream, *first.pct)
        return out.cpu().numpy().astype(np.float64)

    def close(self) -> None:
        for a in self.agents:
            a.close()


class PipelineSource(SnapshotSource):
    """Rank 0 of ``NodePipeline`` (background sampling on every rank)."""

    def __init__(self, pipeline):
        self.pipeline = pipeline
        self._lock = threading.Lock()

    def collect(self):
        with self._lock:
            return self.pipeline.latest_snapshot(), None


class Exporter:
    def __init__(self, source: SnapshotSource, hostname: str | None = None):
        self.source = source
        self.hostname = hostname or socket.gethostname()
        self.scrapes = 0
        self.errors = 0
        self.last_scrape_s = 0.0
        self.scrape_hist = LatencyHistogram("rocmdash_exporter_scrape_latency_seconds", "Collection time per scrape")
        self._server = None

    def render(self) -> str:
        t0 = time.perf_counter()
        try:
            snap, extra = self.source.collect()
            body = render_snapshot(snap, hostname=self.hostname)
            if extra is not None:
                body += extra.text()
        except Exception:
            self.errors += 1
            log.exception("collect failed")
            body = ""
        self.scrapes += 1
        self.last_scrape_s = time.perf_counter() - t0
        self.scrape_hist.observe(self.last_scrape_s)
        own = Exposition()
        self.scrape_hist.add_to(own)
        own.add("rocmdash_exporter_scrapes_total", self.scrapes, {}, "Scrapes served", "counter")
        own.add("rocmdash_exporter_errors_total", self.errors, {}, "Scrapes whose collection failed", "counter")
        own.add("rocmdash_exporter_scrape_seconds", self.last_scrape_s, {}, "Duration of the last collection")
        return body + own.text()

    def health(self) -> tuple:
        """(ok, message) for /healthz: the source's own verdict when it has one (the
        node service reports unhealthy when its refresh loop stalls), else OK."""
        h = getattr(self.source, "health", None)
        if h is None:
            return True, "OK"
        try:
            return h()
        except Exception as e:  # a failing health check is unhealthy, not a 500
            return False, f"health check failed: {e}"

    def serve(self, host: str = "0.0.0.0", port: int = 9400) -> ThreadingHTTPServer:
        exporter = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def do_GET(self):
                if self.path.split("?")[0] == "/metrics":
                    body = exporter.render().encode()
                    ctype = CONTENT_TYPE
                    code = 200
                elif self.path in ("/healthz", "/-/healthy"):
                    ok, msg = exporter.health()
                    body, ctype, code = (msg + "\n").encode(), "text/plain", 200 if ok else 503
                else:
                    body, ctype, code = b"not found\n", "text/plain", 404
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        srv = ThreadingHTTPServer((host, port), Handler)
        srv.daemon_threads = True
        threading.Thread(target=srv.serve_forever, name="rocmdash-exporter", daemon=True).start()
        self._server = srv
        return srv

    @property
    def port(self) -> int:
        return self._server.server_address[1] if self._server else 0

    def close(self) -> None:
        if self._server is not None:
            self._server.shutdown()
            self._server.server_close()
            self._server = None
        self.source.close()


def main(argv=None) -> int:
    from .. import config

    ap = argparse.ArgumentParser(description="rocmdash node exporter (amd_gpu_* + window statistics)")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=config.EXPORTER_PORT)
    ap.add_argument("--synthetic", type=int, default=0, help="serve a synthetic node with N GPUs")
    ap.add_argument("--source", default="auto", choices=["auto", "hw", "synthetic"])
    ap.add_argument("--counters", default="auto", choices=["auto", "hw", "synthetic", "off"])
    ap.add_argument("--node-window", action="store_true", help="also export node-wide window statistics")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    src = SyntheticSource(args.synthetic) if args.synthetic else LocalNodeSource(source=args.source, counters=args.counters, node_window=args.node_window)
    exp = Exporter(src)
    exp.serve(args.host, args.port)
    log.info("serving /metrics on %s:%d", args.host, exp.port)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        exp.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
