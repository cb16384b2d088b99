"""Node exporter: ``/metrics`` with the ``amd_gpu_*`` series the dashboard queries.

Reference counterpart: the AMD device-metrics exporter the reference assumes is
scraped by Prometheus (``app.py:168-171``; not part of the reference repo). This
exporter is fed by rocmdash's own native pipeline:

  * ``LocalNodeSource``: the single-process exporter (no torchrun): one ``GpuAgent``
    per device with background native samplers (amd-smi 10 Hz, device counters
    100 Hz); a scrape refreshes every agent's device window (one window-stats launch
    per GPU) and renders latest values + per-GPU window statistics. It does no
    node-wide aggregation: the node-window statistics and the whole-node tensor come
    only from the rank-per-GPU service (``rocmdash.serve``, RCCL all-gather), the one
    node-aggregation path;
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

from ..models.health import SourceHealth
from ..models.schema import HEALTH_SOURCES, STAT_INDEX
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

    def __init__(self, devices=None, source: str = "auto", counters: str = "auto", cfg=None):
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
        self._health = np.empty((len(self.agents), len(HEALTH_SOURCES), 8), dtype=np.float32)

    def collect(self):
        import torch

        with self._lock:
            t0 = time.perf_counter()
            outs = [a.refresh() for a in self.agents]  # one launch per GPU, all async
            host = np.stack([o.to("cpu", non_blocking=False).numpy() for o in outs])
            now_ns = time.time_ns()
            for i, a in enumerate(self.agents):
                a.health_rows(self._health[i], now_ns)
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
            xcd=np.stack([a.xcd() for a in self.agents]),
            # same per-source health rows the rank-per-GPU service gathers
            source_health=SourceHealth(self._health.copy(),
                                       [(a.info.smi_backend, a.info.counter_backend) for a in self.agents],
                                       self.agents[0].cfg.stale_periods),
        )
        exp = Exposition()
        for a, gid in zip(self.agents, ids):
            for sampler in a.samplers:
                lab = {"gpu_id": gid, "source": sampler.source.kind, "backend": sampler.source.backend}
                exp.add("rocmdash_sampler_read_seconds", sampler.stats()["mean_us"] * 1e-6, lab,
                        "Mean duration of one source read")
        exp.add("rocmdash_refresh_seconds", self.last_refresh_s, {}, "Device refresh (stats kernel + D2H) of the last scrape")
        self.refresh_hist.add_to(exp)
        torch.cuda.synchronize()
        return snap, exp

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
        self._cached = (None, None, "")  # (snapshot, extra, rendered body) of the last scrape

    def render(self) -> str:
        t0 = time.perf_counter()
        try:
            snap, extra = self.source.collect()
            if snap is self._cached[0] and extra is self._cached[1]:
                body = self._cached[2]  # same refresh as the last scrape (node service: 1 Hz)
            else:
                body = render_snapshot(snap, hostname=self.hostname)
                if extra is not None:
                    body += extra.text()
                self._cached = (snap, extra, body)
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
            # headers and body leave in two writes: without TCP_NODELAY the body waits for
            # the client's delayed ACK of the headers (~40 ms per keep-alive request)
            disable_nagle_algorithm = True

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
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    src = SyntheticSource(args.synthetic) if args.synthetic else LocalNodeSource(source=args.source, counters=args.counters)
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
