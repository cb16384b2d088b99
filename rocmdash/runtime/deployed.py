"""The deployed data path, measured inside a running job (bench.py's ``deployed_path``).

``tools/bench_e2e.py`` measures the deployed chain with a separate world-1 service; this
is the same chain run collectively by the job's OWN ranks, so it measures the path users
see at the job's node size (N = 1..8):

    every rank: background sampling at the production rates (amd-smi 10 Hz, device
      counters 100 Hz) -> the service refresh (``rocmdash.serve.refresh_node``: stats
      kernel -> native RCCL ncclAllGather -> publish kernel, health / footprint rows)
      at ``refresh_hz``
    rank 0: ``/metrics`` (the service's exporter) -> mini-Prometheus scrape every
      ``scrape_s`` -> the page's Prometheus data path (the reference's two instant
      queries, ``app.py:157, 167-172``, + the extended query) -> NodeSnapshot -> the frame
      (4 + 4N figures with the extended panels, tables), serialised

and records per page refresh ``page_ms`` (fetch + snapshot + frame, BASELINE.md's
"full refresh" on live data over real sockets) and the display age of every source's
newest sample (display time - the sample's own time, from
``rocmdash_node_refresh_timestamp_seconds - rocmdash_sample_age_seconds``).

Reference: a fetch every ``REFRESH_INTERVAL`` = 5 s (``app.py:331, 486``), freshness
bounded by an external exporter and scrape interval.
"""

from __future__ import annotations

import random
import statistics
import threading
import time

import numpy as np


def _summary(xs, scale=1.0, nd=3):
    xs = sorted(x for x in xs if x == x)
    if not xs:
        return None
    return {"p50": round(statistics.median(xs) * scale, nd), "p90": round(xs[min(len(xs) - 1, int(0.9 * len(xs)))] * scale, nd),
            "n": len(xs)}


def run_deployed_path(agent, agg, *, seconds: float = 5.0, refresh_hz: float = 10.0, scrape_s: float = 0.25,
                      page_s: float = 0.25, collective_timeout_s: float = 60.0) -> dict | None:
    """Collective (every rank). Returns rank 0's summary, None elsewhere. The agent must
    have no sample request pending; it samples in the background during the run and is
    stopped again afterwards."""
    from ..prom.exporter import Exporter
    from ..prom.mini import MiniPrometheus
    from ..prom.query import PrometheusClient, fetch_node_snapshot
    from ..serve import _Latest, refresh_node
    from ..viz.panels import render_frame_json
    from .footprint import Footprint
    from .pipeline import NodePipeline

    pipe = NodePipeline(agent, agg, device_timing=True, health=True, extended=True,
                        collective_timeout_s=collective_timeout_s)
    pipe.footprint = Footprint(agent.device if agent.use_gpu else None)
    period = 1.0 / refresh_hz
    latest = _Latest(max(10.0, 5 * period))
    root = pipe.is_root
    done = threading.Event()
    rec = {"page_ms": [], "ages": {}, "figures": 0, "payload_bytes": 0, "error": None, "stages": {}}
    exporter = prom = None
    if root:
        exporter = Exporter(latest)
        exporter.serve("127.0.0.1", 0)
        prom = MiniPrometheus(scrape_interval=scrape_s)
        prom.add_target(f"http://127.0.0.1:{exporter.port}/metrics")
        prom.db.add({"__name__": "kube_pod_info", "pod": "prometheus-server-0", "host_ip": "127.0.0.1"}, 1.0)
        prom.serve("127.0.0.1", 0)
        client = PrometheusClient(endpoint=f"http://127.0.0.1:{prom.port}/api/v1/query")

        def page_loop():
            try:
                # the first scrape that carries a refresh
                t_wait = time.monotonic() + 30.0
                while time.monotonic() < t_wait:
                    try:
                        snap = fetch_node_snapshot(client, extended=True)
                        if snap.refresh_time is not None:
                            break
                    except Exception:  # noqa: BLE001 - not scraped yet
                        pass
                    time.sleep(scrape_s / 2)
                render_frame_json(snap, snap.gpu_ids, use_gauge=True, extended=True)  # warm-up
                rng = random.Random(0)
                t_end = time.monotonic() + seconds
                next_t = time.monotonic()
                while not rec["page_ms"] or time.monotonic() < t_end:
                    t0 = time.perf_counter()
                    snap = fetch_node_snapshot(client, extended=True)
                    payload = render_frame_json(snap, snap.gpu_ids, use_gauge=True, extended=True)
                    rec["page_ms"].append((time.perf_counter() - t0) * 1e3)
                    t_display = time.time()
                    if snap.source_health is not None and snap.refresh_time is not None:
                        for st in snap.source_health.statuses():
                            if st.age_s == st.age_s:
                                rec["ages"].setdefault(st.kind, []).append(t_display - (snap.refresh_time - st.age_s))
                    rec["figures"] = payload.count('"data"')
                    rec["payload_bytes"] = len(payload)
                    rec["gpus"] = len(snap.gpu_ids)
                    next_t += page_s * rng.uniform(0.5, 1.5)  # random phase against the refresh / scrape
                    time.sleep(max(0.0, next_t - time.monotonic()))
            except Exception as e:  # noqa: BLE001 - reported in the summary
                rec["error"] = f"{type(e).__name__}: {e}"
            finally:
                done.set()

        page = threading.Thread(target=page_loop, name="rocmdash-page", daemon=True)
    c0, t0_run, cpu0 = agent.sample_counts(), time.perf_counter(), time.process_time()
    agent.start()
    stage_us = {}
    started = False
    try:
        next_t = time.monotonic()
        t_limit = time.monotonic() + seconds + 45.0
        while True:
            pipe.stop_vote = 1.0 if (root and (done.is_set() or time.monotonic() > t_limit)) else 0.0
            votes = refresh_node(pipe, agg, None, latest)
            if root and not started:  # scrape once a refresh exists
                started = True
                prom.start_scraping()
                page.start()
            if root:
                for k, v in pipe.stage_seconds().items():
                    stage_us.setdefault(k, []).append(v * 1e6)
                if pipe.launch_host_s is not None:  # host time inside the stats stage's events
                    stage_us.setdefault("stats_launch_host", []).append(pipe.launch_host_s * 1e6)
            if votes is not None and float(np.nanmax(votes)) >= 1.0:
                break
            next_t += period
            delay = next_t - time.monotonic()
            if delay > 0:
                time.sleep(delay)
            else:
                next_t = time.monotonic()
    finally:
        agent.stop()
        pipe.close()
        if prom is not None:
            prom.close()
        if exporter is not None:
            exporter.close()
    # what the production sampling rates deliver, and what they cost: fresh values per
    # second (the bench's accounting, GpuAgent.fresh_samples) and this process's CPU
    # seconds per second (every thread: samplers, the runtime's poller, RCCL, HTTP)
    wall = time.perf_counter() - t0_run
    mine = (agent.fresh_samples(c0, agent.sample_counts()) / wall, (time.process_time() - cpu0) / wall)
    per_rank = agg.all_gather_object(mine)
    if not root:
        return None
    ages = {k: _summary(v, 1e3, 1) for k, v in rec["ages"].items()}
    page_ms = _summary(rec["page_ms"])
    return {
        "path": "serve refresh (native RCCL gather) -> /metrics -> mini-Prometheus scrape -> the page's 3 instant "
                "queries -> NodeSnapshot -> frame JSON (what users see)",
        "config": {"service_refresh_hz": refresh_hz, "scrape_s": scrape_s, "page_s": page_s, "seconds": seconds,
                   "sampling": f"amd-smi {agent.cfg.smi_hz:g} Hz, counters {agent.cfg.counter_hz:g} Hz"},
        "prometheus_page_ms": page_ms,
        "display_age_ms": ages,
        "figures": rec["figures"],
        "payload_bytes": rec["payload_bytes"],
        "gpus": rec.get("gpus"),
        "service_stage_us_p50": {k: round(statistics.median(v), 2) for k, v in stage_us.items()},
        "gather": pipe.gather_report(),
        "production_fresh_per_s_per_gpu": round(sum(f for f, _ in per_rank) / len(per_rank), 1),
        "production_fresh_per_s_by_rank": [round(f, 1) for f, _ in per_rank],
        "cpu_seconds_per_s_by_rank": [round(c, 4) for _, c in per_rank],
        "error": rec["error"],
    }
