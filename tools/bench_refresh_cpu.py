#!/usr/bin/env python3
"""CPU refresh-latency benchmark of the Prometheus path, reference vs rocmdash.

Reproduces BASELINE.md's methodology: ``requests.get`` is replaced by
a function returning canned Prometheus ``/api/v1/query`` JSON for N GPUs (5
``amd_gpu_*`` series each), all N GPUs are selected, and one refresh is timed as

  reference: fetch_gpu_metrics() + selected-GPU averages (app.py:335-345)
             + 4 + 4N create_visualization(...) + fig.to_json() each
  rocmdash:  fetch_node_snapshot() + build_frame() + Frame.to_json()
             (the same figures, JSON-identical: tests/test_app.py)

40 iterations, first 5 dropped, p50/p90 of the rest. The reference runs behind the
recording Streamlit double (Streamlit is not installed here).

    python tools/bench_refresh_cpu.py [--gpus 1 2 4 8] [--iters 40] [--out file.json]
"""

from __future__ import annotations

import argparse
import importlib.util
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REFERENCE_APP = "/root/reference/app.py"


def canned_get(n_gpus: int, card_model: str):
    from rocmdash.prom.mock import FakeResponse, SyntheticNode, prometheus_response

    node = SyntheticNode(n_gpus, card_model=card_model, seed=n_gpus)
    series = node.series()
    pod = prometheus_response([s for s in series if s[0]["__name__"] == "kube_pod_info"])
    gpu = prometheus_response([s for s in series if s[0]["__name__"] != "kube_pod_info"])

    def get(url=None, params=None, timeout=None, **kw):
        q = params["query"]
        return FakeResponse(pod if q.startswith("kube_pod_info") else gpu)

    return get


def time_it(fn, iters: int, drop: int = 5):
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts = sorted(ts[drop:])
    return statistics.median(ts), ts[min(len(ts) - 1, int(0.9 * len(ts)))]


def reference_refresh_fn(n: int, get):
    sys.path.insert(0, os.path.join(ROOT, "tests", "stubs"))
    import streamlit as st  # the recording double

    spec = importlib.util.spec_from_file_location("reference_app", REFERENCE_APP)
    app = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(app)
    app.requests.get = get
    st.session_state["use_gauge"] = True
    selected = [str(g) for g in range(n)]

    def refresh():
        df, stats = app.fetch_gpu_metrics()
        filtered = df.loc[selected]
        numeric = [c for c in filtered.columns if c != "card_model"]
        averages = filtered[numeric].mean()
        pw = filtered["amd_gpu_average_package_power"]
        nz = pw[pw > 0]
        if not nz.empty:
            averages["amd_gpu_average_package_power"] = nz.mean()
        figs = [
            app.create_visualization(averages.get("amd_gpu_gfx_activity", 0), "Avg GPU Utilization (%)", 100, 300, "k", selected[0], df),
            app.create_visualization(averages.get("vram_usage_ratio", 0), "Avg VRAM Usage (%)", 100, 300, "k"),
            app.create_visualization(averages.get("amd_gpu_edge_temperature", 0), "Avg Temperature (°C)", 100, 300, "k"),
            app.create_visualization(averages.get("amd_gpu_average_package_power", 0), "Avg Power Usage (W)", 300, 300, "k", selected[0], df),
        ]
        for gid, m in filtered.iterrows():
            figs.append(app.create_visualization(m.get("amd_gpu_gfx_activity", 0), "GPU Utilization (%)", 100, 200, "k", gid, df))
            figs.append(app.create_visualization(m.get("vram_usage_ratio", 0), "VRAM Usage (%)", 100, 200, "k", gid, df))
            figs.append(app.create_visualization(m.get("amd_gpu_edge_temperature", 0), "Temperature (°C)", 100, 200, "k", gid, df))
            figs.append(app.create_visualization(m.get("amd_gpu_average_package_power", 0), "Power Usage (W)", 300, 200, "k", gid, df))
        for f in figs:
            f.to_json()
        st.CALLS.clear()
        return len(figs)

    return refresh


def ours_refresh_fn(n: int, get):
    from rocmdash.prom.query import PrometheusClient, fetch_node_snapshot
    from rocmdash.viz.panels import build_frame

    client = PrometheusClient(endpoint="http://prom/api/v1/query", get=get)

    def refresh():
        snap = fetch_node_snapshot(client)
        frame = build_frame(snap, snap.gpu_ids)
        frame.to_json()
        return frame.num_figures

    return refresh


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--card-model", default="102-G30211-0C")
    ap.add_argument("--no-reference", action="store_true")
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    rows = []
    for n in args.gpus:
        get = canned_get(n, args.card_model)
        ours = ours_refresh_fn(n, get)
        assert ours() == 4 + 4 * n
        o50, o90 = time_it(ours, args.iters)
        row = {"n_gpus": n, "figures": 4 + 4 * n, "rocmdash_p50_ms": round(o50, 3), "rocmdash_p90_ms": round(o90, 3)}
        if not args.no_reference and os.path.exists(REFERENCE_APP):
            ref = reference_refresh_fn(n, get)
            assert ref() == 4 + 4 * n
            r50, r90 = time_it(ref, args.iters)
            row.update(reference_p50_ms=round(r50, 3), reference_p90_ms=round(r90, 3), speedup_p50=round(r50 / o50, 1))
        rows.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"method": "BASELINE.md / SURVEY.md §6 (canned Prometheus JSON, all GPUs selected)", "rows": rows}, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
