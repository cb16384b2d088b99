#!/usr/bin/env python3
"""End-to-end benchmark of the DEPLOYED data path: how old is a sample when the page
shows it, and how long does a page refresh take?

    rocmdash.serve (world 1, live amd-smi 10 Hz + device counters 100 Hz, refresh
      --refresh-hz) -> /metrics -> mini-Prometheus scrape every --scrape-s
      -> the page's Prometheus data path: the reference's two instant queries
         (app.py:157, 167-172) + the one extended query -> NodeSnapshot
      -> the frame (4 + 4N figures + tables, extended panels), serialised

and the page's ``native`` mode (one scrape of the service's /metrics, no
Prometheus). bench.py measures the closed loop (sample -> stats -> frame as fast as
the hardware allows); this is the production configuration of the same chain
(reference: a fetch at ``app.py:331`` every ``REFRESH_INTERVAL`` = 5 s, ``app.py:486``).

Per page refresh it records:
  * ``page_ms``: fetch (HTTP queries) + snapshot + frame JSON, the BASELINE.md
    "full refresh" definition on live data over real sockets;
  * ``age_s[source]``: display time - the sample's own time, where the sample's time
    is ``rocmdash_node_refresh_timestamp_seconds - rocmdash_sample_age_seconds``
    (both exported by the service and read in the page's own snapshot: they come from
    the same scrape). It adds up the
    sampler period, the service refresh period, the scrape interval and the query.

    python tools/bench_e2e.py [--seconds 40] [--refresh-hz 1] [--scrape-s 1]
        [--page-s 1] [--out file.json] [--cpu]   (--cpu: synthetic sources, gloo)
    python tools/bench_e2e.py --manifests deploy/k8s [--seconds 40]

``--manifests``: the DaemonSet configuration as deployed - the service's flags
(``--refresh-hz``, ``--node-window``) and env come from exporter-daemonset.yaml, the page's
env (``ROCMDASH_EXTENDED`` ...) from dashboard.yaml (only the endpoint is local), so the
page renders exactly the panel set the manifests ship (world size 1 on a 1-GPU box: the
DaemonSet runs one rank per GPU). The scrape interval is prometheus.yaml's.
"""

from __future__ import annotations

import argparse
import json
import os
import random
import signal
import socket
import statistics
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pct(xs, q):
    xs = sorted(x for x in xs if x == x)
    if not xs:
        return None
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def _summary(xs, scale=1.0, nd=4):
    xs = [x for x in xs if x == x]
    if not xs:
        return None
    return {"p50": round(statistics.median(xs) * scale, nd), "p90": round(_pct(xs, 0.9) * scale, nd),
            "max": round(max(xs) * scale, nd), "n": len(xs)}


def _wait_ready(url: str, proc, timeout: float) -> None:
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if proc.poll() is not None:
            raise RuntimeError(f"node service exited with {proc.returncode}")
        try:
            with urllib.request.urlopen(url, timeout=2) as r:
                if r.status == 200 and b"rocmdash_node_refresh_timestamp_seconds" in r.read():
                    return
        except OSError:
            pass
        time.sleep(0.25)
    raise RuntimeError(f"node service not ready at {url} within {timeout} s")


def _ages(snap, refresh_ts: float, t_display: float) -> dict:
    """Display age of the newest sample of every source of every GPU (seconds)."""
    out = {}
    if snap.source_health is None:
        return out
    for st in snap.source_health.statuses():
        if st.age_s == st.age_s:
            out.setdefault(st.kind, []).append(t_display - (refresh_ts - st.age_s))
    return out


def _from_manifests(path: str) -> dict:
    """Service flags / env, page env and scrape interval from the K8s manifests."""
    import yaml

    docs = []
    for fn in ("exporter-daemonset.yaml", "dashboard.yaml", "prometheus.yaml"):
        with open(os.path.join(path, fn)) as f:
            docs += [d for d in yaml.safe_load_all(f) if d]
    by = {(d["kind"], d["metadata"]["name"]): d for d in docs}
    ds = by[("DaemonSet", "rocmdash-exporter")]["spec"]["template"]["spec"]["containers"][0]
    dash = by[("Deployment", "rocmdash-dashboard")]["spec"]["template"]["spec"]["containers"][0]
    args = ds["args"][ds["args"].index("rocmdash.serve") + 1:]
    hz = [a.split("=", 1)[1] for a in args if a.startswith("--refresh-hz=")]
    prom = yaml.safe_load(by[("ConfigMap", "prometheus-config")]["data"]["prometheus.yml"])
    job = {j["job_name"]: j for j in prom["scrape_configs"]}["amd-gpu-exporter"]
    interval = job.get("scrape_interval", prom.get("global", {}).get("scrape_interval", "15s"))
    return {
        "refresh_hz": float(hz[0]) if hz else 1.0,
        "node_window": "--node-window" in args,
        "serve_env": {e["name"]: e["value"] for e in ds.get("env", []) if e["name"] != "HSA_ENABLE_IPC_MODE_LEGACY"},
        "page_env": {e["name"]: e["value"] for e in dash.get("env", [])},
        "scrape_s": float(interval.rstrip("s")),
    }


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--seconds", type=float, default=40.0, help="measurement time per data path")
    ap.add_argument("--refresh-hz", type=float, default=1.0, help="node service refresh rate (DaemonSet: 1)")
    ap.add_argument("--scrape-s", type=float, default=1.0, help="mini-Prometheus scrape interval")
    ap.add_argument("--page-s", type=float, default=1.0,
                    help="page refresh period (the reference sleeps 5 s; the age is sampled at display time, so a "
                    "shorter period only gives more samples)")
    ap.add_argument("--node-window", action="store_true", help="service exports node-wide window statistics")
    ap.add_argument("--cpu", action="store_true", help="synthetic sources on the CPU (no GPU)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--manifests", default=None, help="take service flags / env and page env from these K8s manifests")
    ap.add_argument("--world", type=int, default=1,
                    help="service ranks (torchrun); more than the box's GPUs runs them oversubscribed (rehearsal of an "
                    "N-GPU node's page on fewer GPUs: RCCL over sockets, counters synthetic)")
    args = ap.parse_args(argv)
    serve_env, manifest = {}, None
    if args.manifests:
        manifest = _from_manifests(args.manifests)
        args.refresh_hz = manifest["refresh_hz"]
        args.node_window = manifest["node_window"]
        args.scrape_s = manifest["scrape_s"]
        serve_env = manifest["serve_env"]
        for k, v in manifest["page_env"].items():
            if k != "PROMETHEUS_METRICS_ENDPOINT":
                os.environ[k] = v
    from rocmdash.prom.query import extended_enabled

    extended = extended_enabled() if manifest else True

    from rocmdash.prom.mini import MiniPrometheus
    from rocmdash.prom.query import PrometheusClient, fetch_node_snapshot, fetch_service_snapshot
    from rocmdash.viz.panels import render_frame_json

    port = _free_port()
    serve = ["-m", "rocmdash.serve", "--host", "127.0.0.1", "--port", str(port), "--refresh-hz", str(args.refresh_hz)]
    if args.cpu:
        serve += ["--cpu", "--source", "synthetic", "--counters", "synthetic"]
    elif args.world > 1:
        serve += ["--counters", "synthetic"]  # one counting context per GPU: the ranks share one here
    if args.node_window:
        serve.append("--node-window")
    env = dict(os.environ, PYTHONPATH=ROOT, **serve_env)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)  # the service (or torchrun) sets up its own environment
    if args.world > 1:  # rank per GPU; more ranks than GPUs: oversubscribed (RCCL over sockets)
        import torch

        if args.cpu or torch.cuda.device_count() < args.world:
            env["ROCMDASH_OVERSUBSCRIBE"] = "1"
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.world),
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *serve]
    else:
        cmd = [sys.executable, *serve]
    log_path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"bench_e2e_serve_{port}.log")
    log = open(log_path, "w")
    proc = subprocess.Popen(cmd, cwd=ROOT, stdout=log, stderr=subprocess.STDOUT, env=env, start_new_session=True)
    metrics_url = f"http://127.0.0.1:{port}/metrics"
    prom = MiniPrometheus(scrape_interval=args.scrape_s)
    result = {}
    try:
        _wait_ready(metrics_url, proc, timeout=300)
        prom.add_target(metrics_url)
        prom.db.add({"__name__": "kube_pod_info", "pod": "prometheus-server-0", "host_ip": "127.0.0.1"}, 1.0)
        if 2 * args.seconds > 250:  # the discovery series must stay inside the 5 min lookback
            raise SystemExit("--seconds: at most 125")
        prom.start_scraping()
        prom.serve("127.0.0.1", 0)
        client = PrometheusClient(endpoint=f"http://127.0.0.1:{prom.port}/api/v1/query")
        time.sleep(max(2 * args.scrape_s, 1.0))

        def prom_page():
            snap = fetch_node_snapshot(client, extended=extended)
            payload = render_frame_json(snap, snap.gpu_ids, use_gauge=True, extended=extended)
            return snap, payload

        def native_page():
            snap = fetch_service_snapshot(metrics_url)
            payload = render_frame_json(snap, snap.gpu_ids, use_gauge=True, extended=extended)
            return snap, payload

        rng = random.Random(0)
        for mode, page in (("prometheus", prom_page), ("native", native_page)):
            page_ms, ages, figs, nbytes = [], {}, 0, 0
            snap, _ = page()  # warm-up: first connection, frame layout compiled once per GPU set
            t_end = time.monotonic() + args.seconds
            next_t = time.monotonic()
            while not page_ms or time.monotonic() < t_end:
                t0 = time.perf_counter()
                snap, payload = page()
                t1 = time.perf_counter()
                t_display = time.time()
                page_ms.append((t1 - t0) * 1e3)
                if snap.refresh_time is None:
                    raise RuntimeError("the snapshot carries no rocmdash_node_refresh_timestamp_seconds")
                for k, v in _ages(snap, snap.refresh_time, t_display).items():
                    ages.setdefault(k, []).extend(v)
                nbytes = len(payload)
                figs = payload.count('"data"')
                # random phase against the service and scrape periods (no lock-step)
                next_t += args.page_s * rng.uniform(0.5, 1.5)
                time.sleep(max(0.0, next_t - time.monotonic()))
            result[mode] = {
                "page_ms": _summary(page_ms, nd=3),
                "display_age_ms": {k: _summary(v, 1e3, 1) for k, v in ages.items()},
                "gpus": len(snap.gpu_ids),
                "columns": len(snap.columns),
                "window_series": len(snap.window_series),
                "payload_bytes": nbytes,
                "figures": figs,
            }
            print(json.dumps({mode: result[mode]}), flush=True)
        scrape = [t.last_scrape_s for t in prom.targets]
        result["config"] = {
            "service_refresh_hz": args.refresh_hz, "scrape_s": args.scrape_s, "page_s": args.page_s,
            "node_window": args.node_window, "sources": "synthetic (CPU)" if args.cpu else ("live amd-smi + synthetic counters" if args.world > 1
                                                             else "live amd-smi + rocprofiler"),
            "page_extended": extended, "from_manifests": args.manifests, "service_ranks": args.world,
            "oversubscribed": env.get("ROCMDASH_OVERSUBSCRIBE") == "1",
            "last_scrape_ms": round(scrape[0] * 1e3, 2) if scrape else None,
            "reference": "fetch every 5 s (app.py:331, 486); freshness bounded by the external exporter + scrape",
        }
    finally:
        prom.close()
        if proc.poll() is None:
            os.killpg(proc.pid, signal.SIGTERM)
            try:
                proc.wait(timeout=60)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
                proc.wait()
        log.close()
    line = json.dumps(result)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
