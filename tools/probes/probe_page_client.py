"""Probe: where a page refresh through Prometheus spends its time (rocmdash/prom/query.py
``KeepAliveGet``, rocmdash/prom/mini.py ``query_json``).

Starts ``rocmdash.serve`` with ``--world`` ranks on the CPU (synthetic sources, gloo;
``--node-window``), scrapes it once into a mini-Prometheus, stops the service (no
contention with the measurement), then times the page's parts:
  fetch      the page's three instant queries + NodeSnapshot (query.fetch_node_snapshot)
  render     the frame (4 + 4N figures + extended panels) to JSON
  server     the mini-Prometheus answering the extended query (query_json)
  decode     json.loads of that answer on the client
  snapshot   snapshot_from_series of its series
and prints one JSON line.

    python tools/probes/probe_page_client.py [--world 8]
"""

import argparse
import json
import os
import signal
import socket
import statistics
import subprocess
import sys
import time
import timeit
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    args = ap.parse_args()
    port = _free_port()
    serve = ["-m", "rocmdash.serve", "--cpu", "--source", "synthetic", "--counters", "synthetic", "--port", str(port),
             "--refresh-hz", "1", "--host", "127.0.0.1", "--node-window"]
    cmd = [sys.executable, *serve] if args.world == 1 else [
        sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.world),
        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *serve]
    proc = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                            env=dict(os.environ, PYTHONPATH=ROOT), start_new_session=True)
    from rocmdash.prom.mini import MiniPrometheus
    from rocmdash.prom.query import PrometheusClient, fetch_node_snapshot
    from rocmdash.prom.snapshot_io import extended_query, snapshot_from_series
    from rocmdash.viz.panels import render_frame_json

    try:
        for _ in range(240):
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=2) as r:
                    if b"rocmdash_node_refresh_timestamp_seconds" in r.read():
                        break
            except OSError:
                pass
            time.sleep(0.5)
        prom = MiniPrometheus(scrape_interval=1.0)
        prom.add_target(f"http://127.0.0.1:{port}/metrics")
        prom.db.add({"__name__": "kube_pod_info", "pod": "prometheus-server-0", "host_ip": "127.0.0.1"}, 1.0)
        prom.scrape_all()
    finally:
        os.killpg(proc.pid, signal.SIGTERM)
        proc.wait(timeout=60)
    prom.serve("127.0.0.1", 0)
    client = PrometheusClient(endpoint=f"http://127.0.0.1:{prom.port}/api/v1/query")
    fetch, render = [], []
    for _ in range(25):
        t0 = time.perf_counter()
        snap = fetch_node_snapshot(client, extended=True)
        t1 = time.perf_counter()
        payload = render_frame_json(snap, snap.gpu_ids, use_gauge=True, extended=True)
        render.append((time.perf_counter() - t1) * 1e3)
        fetch.append((t1 - t0) * 1e3)
    q = extended_query("127.0.0.1")
    prom.query(q)
    body = prom.query_json(q)
    items = [(r["metric"], r["value"][1]) for r in json.loads(body)["data"]["result"]]

    def best(fn):
        return round(min(timeit.repeat(fn, number=5, repeat=5)) / 5 * 1e3, 3)

    out = {"world": args.world, "gpus": len(snap.gpu_ids), "series_in_tsdb": prom.db.series_count(),
           "figures": payload.count('"data"'), "extended_answer_bytes": len(body),
           "fetch_ms_p50": round(statistics.median(fetch), 3), "render_ms_p50": round(statistics.median(render), 3),
           "server_ms": best(lambda: prom.query_json(q)), "decode_ms": best(lambda: json.loads(body)),
           "snapshot_ms": best(lambda: snapshot_from_series(items, require_vram=False))}
    prom.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
