"""GPU end-to-end services on one MI355X: the node exporter over live amd-smi (+ the
window-stats kernel) scraped by the mini-Prometheus and read back through the
reference's queries, the rank-per-GPU service (world size 1, RCCL), and the
Streamlit page in native mode."""

import json
import os
import subprocess
import sys
import urllib.request

import pytest

from rocmdash.viz.panels import EXTENDED_PANELS

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_local_node_exporter_scrape_and_reference_query(native):
    from rocmdash.config import SamplerConfig
    from rocmdash.prom.exporter import Exporter, LocalNodeSource
    from rocmdash.prom.exposition import parse_text
    from rocmdash.prom.mini import MiniPrometheus
    from rocmdash.prom.query import PrometheusClient, fetch_gpu_metrics

    src = LocalNodeSource(devices=[0], counters="off", cfg=SamplerConfig(window=1024, ring_capacity=4096, smi_hz=100),
                          node_window=True)
    exp = Exporter(src, hostname="mi355x-box")
    exp.serve("127.0.0.1", 0)
    prom = MiniPrometheus()
    try:
        import time

        time.sleep(0.5)  # ~50 amd-smi samples at 100 Hz
        with urllib.request.urlopen(f"http://127.0.0.1:{exp.port}/metrics") as r:
            body = r.read().decode()
        samples = parse_text(body)
        names = {s.name for s in samples}
        assert {"amd_gpu_gfx_activity", "amd_gpu_total_vram", "rocmdash_window", "rocmdash_source_stale"} <= names
        stale = [s.value for s in samples if s.name == "rocmdash_source_stale"]
        assert stale and all(v == 0 for v in stale), stale
        counts = [s.value for s in samples if s.name == "rocmdash_window_samples"]
        assert counts and min(counts) >= 10
        # node-wide window statistics of one GPU: the union is that GPU's window
        node = {(s.label_dict()["metric"], s.label_dict()["stat"]): s.value for s in samples
                if s.name == "rocmdash_node_window"}
        assert node[("amd_gpu_total_vram", "count")] >= 10 and node[("amd_gpu_total_vram", "min")] > 200_000
        prom.add_target(f"http://127.0.0.1:{exp.port}/metrics")
        prom.db.add({"__name__": "kube_pod_info", "pod": "prometheus-server-0", "host_ip": "127.0.0.1"}, 1.0)
        prom.scrape_all()
        prom.serve("127.0.0.1", 0)
        df, stats = fetch_gpu_metrics(PrometheusClient(endpoint=f"http://127.0.0.1:{prom.port}/api/v1/query"),
                                      on_error=pytest.fail)
        assert len(df) == 1 and df["amd_gpu_total_vram"].iloc[0] > 200_000
        assert df["card_model"].iloc[0].startswith("102-")
    finally:
        prom.close()
        exp.close()


def test_serve_world1_writes_frame_and_metrics(tmp_path):
    frame = tmp_path / "frame.json"
    cmd = [sys.executable, "-m", "rocmdash.serve", "--port", "0", "--refresh-hz", "20", "--max-refreshes", "10",
           "--frame-out", str(frame)]
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    d = json.loads(frame.read_text())
    assert len(d["figures"]) == 4 + 4 + len(EXTENDED_PANELS)  # extended: + MFMA, HBM read/write, xGMI recv/send
    assert d["window"]["series"][0] == "amd_gpu_edge_temperature"


def test_page_native_mode_on_gpu(monkeypatch):
    # HIP is initialised in this pytest process already: counters cannot be
    # registered any more (they need to precede HSA init), so leave them off.
    monkeypatch.setenv("ROCMDASH_COUNTERS", "0")
    monkeypatch.syspath_prepend(os.path.join(ROOT, "tests", "stubs"))
    sys.modules.pop("streamlit", None)
    import importlib.util

    import streamlit as st

    st.reset()
    spec = importlib.util.spec_from_file_location("rocmdash_app_gpu", os.path.join(ROOT, "app.py"))
    app = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(app)
    from rocmdash.ui import page

    page._DataSource._native_agents = None
    st.reset()
    app.main(max_refreshes=2, data_source="native")
    charts = st.calls("plotly_chart")
    assert len(charts) == 2 * (4 + 4)
    headers = [c[1][0] for c in st.calls("markdown") if str(c[1][0]).startswith("###")]
    assert headers and "(MI355X)" in headers[0], headers
    page._DataSource._native_agents.close()
    page._DataSource._native_agents = None
    sys.modules.pop("streamlit", None)
