"""The deployed data path on the CPU, end to end over real sockets:

  rocmdash.serve (rank-per-GPU node service, synthetic sources, gloo)
    -> /metrics -> mini-Prometheus scrape -> the reference's two queries (+ the one
    extended query with ROCMDASH_EXTENDED=1) -> the Streamlit page (test double);

plus the page's ``native`` mode reading the node service directly, and per-rank
source health: a rank whose samplers stall is reported stale by rank 0.
Reference: ``app.py:153-227`` (fetch), ``app.py:412-476`` (per-GPU panels)."""

import os
import signal
import socket
import subprocess
import sys
import time
import urllib.error
import urllib.request

import pytest

from rocmdash.models.schema import CTR_FIELDS, SMI_FIELDS

from rocmdash.viz.panels import EXTENDED_PANELS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _get(url, timeout=2.0):
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.status, r.read().decode()
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode()
    except (urllib.error.URLError, ConnectionError, OSError):
        return None, ""


def _wait_metrics(port, pred=lambda body: True, timeout=90.0):
    deadline = time.monotonic() + timeout
    body = ""
    while time.monotonic() < deadline:
        code, body = _get(f"http://127.0.0.1:{port}/metrics")
        if code == 200 and pred(body):
            return body
        time.sleep(0.2)
    raise AssertionError(f"no matching /metrics on port {port} within {timeout} s; last body:\n{body[-2000:]}")


@pytest.fixture
def node_service():
    """Start ``rocmdash.serve`` (world 1, CPU, synthetic sources, --node-window)."""
    procs = []

    def start(*extra, env=None):
        port = _free_port()
        cmd = [sys.executable, "-m", "rocmdash.serve", "--cpu", "--source", "synthetic", "--counters", "synthetic",
               "--port", str(port), "--refresh-hz", "20", *extra]
        p = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                             env=dict(os.environ, PYTHONPATH=ROOT, **(env or {})), start_new_session=True)
        procs.append(p)
        _wait_metrics(port, lambda b: "rocmdash_window{" in b)
        return port

    yield start
    for p in procs:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGTERM)
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()


def _run_page(st_stub, monkeypatch, data_source, **env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    from rocmdash import config

    config.reload()
    import importlib.util

    spec = importlib.util.spec_from_file_location("rocmdash_app_deployed", os.path.join(ROOT, "app.py"))
    app = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(app)
    st_stub.reset()
    app.main(max_refreshes=1, data_source=data_source)
    errors = st_stub.calls("error")
    assert not errors, errors
    return st_stub


def _chart_keys(st):
    return [c[2]["key"] for c in st.calls("plotly_chart")]


def test_extended_panels_through_prometheus(node_service, st_stub, monkeypatch):
    """ROCMDASH_EXTENDED=1 in Prometheus mode: the page shows the MFMA / HBM / xGMI
    gauges and the windowed-statistics table from the node service's export, read
    through the mini-Prometheus with the reference's queries + one extended query."""
    from rocmdash.prom.mini import MiniPrometheus

    port = node_service("--node-window")
    prom = MiniPrometheus()
    try:
        prom.add_target(f"http://127.0.0.1:{port}/metrics")
        prom.db.add({"__name__": "kube_pod_info", "pod": "prometheus-server-0", "host_ip": "127.0.0.1"}, 1.0)
        prom.scrape_all()
        prom.serve("127.0.0.1", 0)
        endpoint = f"http://127.0.0.1:{prom.port}/api/v1/query"
        st = _run_page(st_stub, monkeypatch, "prometheus", PROMETHEUS_METRICS_ENDPOINT=endpoint, ROCMDASH_EXTENDED="1")
        keys = _chart_keys(st)
        assert len(keys) == 4 + 4 + len(EXTENDED_PANELS), keys
        for _, _, key, _ in EXTENDED_PANELS:
            assert any(k.startswith(f"plot_{key}_0_") for k in keys), (key, keys)
        subs = [c[1][0] for c in st.calls("subheader")]
        assert "Windowed Statistics (HIP window-stats kernel)" in subs, subs
        assert "Node-wide Windowed Statistics (all GPUs)" in subs, subs
        assert "Per-XCD Activity and Clocks" in subs  # the synthetic SMU source models 8 XCDs

        # the compat contract is untouched by the extended query
        from rocmdash.prom.query import PrometheusClient, fetch_gpu_metrics

        df, stats = fetch_gpu_metrics(PrometheusClient(endpoint=endpoint), on_error=pytest.fail)
        assert set(df.columns) == {"amd_gpu_edge_temperature", "amd_gpu_gfx_activity",
                                   "amd_gpu_average_package_power", "amd_gpu_used_vram", "amd_gpu_total_vram",
                                   "card_model", "vram_usage_ratio"}
    finally:
        prom.close()


def _manifest_env(kind, name):
    import yaml

    with open(os.path.join(ROOT, "deploy", "k8s", "dashboard.yaml" if kind == "Deployment" else
                           "exporter-daemonset.yaml")) as f:
        for d in yaml.safe_load_all(f):
            if d and d["kind"] == kind and d["metadata"]["name"] == name:
                c = d["spec"]["template"]["spec"]["containers"][0]
                return {e["name"]: e["value"] for e in c.get("env", [])}, c.get("args", [])
    raise AssertionError(f"{kind}/{name} not in the manifests")


def test_manifest_dashboard_env_shows_the_multi_panel_view(node_service, st_stub, monkeypatch):
    """The page as DEPLOYED: every env var of deploy/k8s/dashboard.yaml (only the
    Prometheus endpoint redirected to the local mini-Prometheus) against the node service
    started with the DaemonSet's flags. The page must show the extended panels and
    tables - the multi-panel view of BASELINE.json config #5 - not just the reference's
    five panels; drop ROCMDASH_EXTENDED from the manifest and this fails."""
    from rocmdash.prom.mini import MiniPrometheus

    env, _ = _manifest_env("Deployment", "rocmdash-dashboard")
    _, ds_args = _manifest_env("DaemonSet", "rocmdash-exporter")
    serve_flags = [a for a in ds_args[ds_args.index("rocmdash.serve") + 1:] if a == "--node-window"]
    port = node_service(*serve_flags)
    prom = MiniPrometheus()
    try:
        prom.add_target(f"http://127.0.0.1:{port}/metrics")
        prom.db.add({"__name__": "kube_pod_info", "pod": env["PROMETHEUS_METRICS_PODNAME"] + "-0",
                     "host_ip": "127.0.0.1"}, 1.0)
        prom.scrape_all()
        prom.serve("127.0.0.1", 0)
        monkeypatch.delenv("ROCMDASH_EXTENDED", raising=False)
        env = dict(env, PROMETHEUS_METRICS_ENDPOINT=f"http://127.0.0.1:{prom.port}/api/v1/query")
        st = _run_page(st_stub, monkeypatch, "prometheus", **env)
        keys = _chart_keys(st)
        assert len(keys) == 4 + 4 + len(EXTENDED_PANELS), keys
        subs = [c[1][0] for c in st.calls("subheader")]
        assert "Windowed Statistics (HIP window-stats kernel)" in subs, subs
        assert "Node-wide Windowed Statistics (all GPUs)" in subs, subs
    finally:
        prom.close()


def test_extended_snapshot_matches_service(node_service):
    """The snapshot rebuilt from the Prometheus query equals the one read straight
    from the service's exposition: same columns, window statistics and health."""
    import numpy as np

    from rocmdash.prom.mini import MiniPrometheus
    from rocmdash.prom.query import PrometheusClient, fetch_node_snapshot, fetch_service_snapshot

    port = node_service("--node-window")
    prom = MiniPrometheus()
    try:
        prom.add_target(f"http://127.0.0.1:{port}/metrics")
        prom.db.add({"__name__": "kube_pod_info", "pod": "prometheus-server-0", "host_ip": "127.0.0.1"}, 1.0)
        # scrape and read the service within one refresh period of each other
        prom.scrape_all()
        direct = fetch_service_snapshot(f"http://127.0.0.1:{port}/metrics")
        prom.serve("127.0.0.1", 0)
        snap = fetch_node_snapshot(PrometheusClient(endpoint=f"http://127.0.0.1:{prom.port}/api/v1/query"),
                                   extended=True)
    finally:
        prom.close()
    assert snap.gpu_ids == ["0"] and direct.gpu_ids == ["0"]
    for col in ("amd_gpu_mfma_utilization", "amd_gpu_hbm_read_bandwidth", "amd_gpu_xgmi_read_bandwidth"):
        assert snap.has(col) and direct.has(col)
    assert snap.window is not None and snap.window.shape == (1, len(SMI_FIELDS) + len(CTR_FIELDS), 8)
    assert snap.window_series == direct.window_series
    assert snap.node_window is not None and snap.node_window.shape == (len(SMI_FIELDS) + len(CTR_FIELDS), 8)
    # counts of the windowed samples are integers > 0 on both paths
    assert (snap.window[0, :, 7] > 0).all() and np.all(snap.window[0, :, 7] == np.round(snap.window[0, :, 7]))
    assert snap.source_health is not None
    st = {s.kind: s for s in snap.source_health.statuses()}
    assert set(st) == {"smi", "counter"} and not any(s.stale for s in st.values())
    assert st["counter"].samples > 0 and st["counter"].backend == "synthetic"


def test_page_native_mode_reads_node_service(node_service, st_stub, monkeypatch):
    """``native`` mode: the page scrapes the rank-per-GPU service directly - the node
    view it shows is the gathered node tensor (no peer copies, no Prometheus)."""
    port = node_service("--node-window")
    st = _run_page(st_stub, monkeypatch, "native", ROCMDASH_NODE_ENDPOINT=f"http://127.0.0.1:{port}/metrics",
                   ROCMDASH_EXTENDED="1")
    keys = _chart_keys(st)
    assert len(keys) == 4 + 4 + len(EXTENDED_PANELS), keys
    subs = [c[1][0] for c in st.calls("subheader")]
    assert "Node-wide Windowed Statistics (all GPUs)" in subs


def test_serve_reports_stalled_rank_stale():
    """Per-rank health on the deployed path: 2 gloo ranks, rank 1's samplers stop
    after 3 refreshes (it keeps refreshing and answering collectives). Rank 0's
    /metrics turns rocmdash_source_stale{gpu_id="1"} to 1 while GPU 0 stays 0, and
    /healthz stays 200 naming the stale source (liveness follows the refresh loop only:
    VERDICT r04 weak 1)."""
    from rocmdash.prom.exposition import parse_text

    port = _free_port()
    mport = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(mport),
           "-m", "rocmdash.serve", "--cpu", "--source", "synthetic", "--counters", "synthetic", "--port", str(port),
           "--refresh-hz", "20", "--max-refreshes", "600", "--collective-timeout", "20"]
    env = dict(os.environ, ROCMDASH_FAULT="stall:1:3", PYTHONPATH=ROOT)
    p = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env,
                         start_new_session=True)
    try:
        def stale_of(body):
            out = {}
            for s in parse_text(body):
                if s.name == "rocmdash_source_stale":
                    d = s.label_dict()
                    out[(d["gpu_id"], d["source"])] = s.value
            return out

        # the stall's effect, not a start-up transient (under load a rank's first rows can
        # arrive late): GPU 0 fresh, GPU 1 stale, and the fault injection logged
        t_first = []

        def settled(b):
            st = stale_of(b)
            ok = st.get(("1", "smi")) == 1.0 and st.get(("0", "smi")) == 0.0 and st.get(("0", "counter")) == 0.0
            if ok and not t_first:
                t_first.append(time.monotonic())
            return ok and time.monotonic() - t_first[0] > 1.0 and stale_of(b).get(("1", "smi")) == 1.0

        body = _wait_metrics(port, settled, timeout=120)
        st = stale_of(body)
        assert st[("1", "smi")] == 1.0 and st[("1", "counter")] == 1.0, st
        assert st[("0", "smi")] == 0.0 and st[("0", "counter")] == 0.0, st
        code, msg = _get(f"http://127.0.0.1:{port}/healthz")
        assert code == 200 and "gpu 1" in msg and "stale" in msg, (code, msg)
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGTERM)
        out, _ = p.communicate(timeout=60)
    assert "fault injection: rank 1 stall" in out, out[-3000:]


def test_bench_e2e_tool_on_cpu(tmp_path):
    """tools/bench_e2e.py end to end on the CPU: node service (synthetic sources) ->
    mini-Prometheus -> page in both data-source modes; every page carries the refresh
    time, so each displayed sample's age is known and bounded by the periods."""
    import json

    out = tmp_path / "e2e.json"
    res = subprocess.run([sys.executable, "tools/bench_e2e.py", "--cpu", "--seconds", "4", "--refresh-hz", "4",
                          "--scrape-s", "0.25", "--page-s", "0.3", "--out", str(out)],
                         cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    d = json.loads(out.read_text())
    for mode in ("prometheus", "native"):
        m = d[mode]
        assert m["page_ms"]["n"] >= 5 and m["figures"] >= 4 + 4 + len(EXTENDED_PANELS), m  # + the tables
        ages = m["display_age_ms"]
        assert set(ages) == {"smi", "counter"}, ages
        # service period 250 ms + scrape 250 ms (+ query): a displayed sample is < 2 s old
        assert 0 < ages["counter"]["p50"] < 2000 and ages["counter"]["max"] < 5000, ages
    assert d["config"]["sources"].startswith("synthetic")


def test_serve_exports_every_ranks_footprint():
    """Every rank's own cost rides in its control row of the ONE gather: rank 0 exports
    rocmdash_self_rss_bytes / rocmdash_self_cpu_seconds_total (a counter that grows)
    for BOTH ranks of a 2-rank gloo service, plus the gather state of each rank."""
    from rocmdash.prom.exposition import parse_text

    port, mport = _free_port(), _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(mport),
           "-m", "rocmdash.serve", "--cpu", "--source", "synthetic", "--counters", "synthetic", "--port", str(port),
           "--refresh-hz", "20", "--max-refreshes", "400", "--collective-timeout", "20"]
    p = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                         env=dict(os.environ, PYTHONPATH=ROOT), start_new_session=True)
    try:
        def self_of(body):
            out = {}
            for s in parse_text(body):
                if s.name.startswith("rocmdash_self_") or s.name.startswith("rocmdash_gather_"):
                    d = s.label_dict()
                    out[(s.name + (":" + d["class"] if "class" in d else ""), d.get("gpu_id"))] = s.value
            return out

        body = _wait_metrics(port, lambda b: ("rocmdash_self_cpu_seconds_total:normal", "1") in self_of(b), timeout=120)
        a = self_of(body)
        time.sleep(1.0)
        b = self_of(_wait_metrics(port))
        for g in ("0", "1"):
            assert a[("rocmdash_self_rss_bytes", g)] > 50 * 2**20, a
            k = "rocmdash_self_cpu_seconds_total:normal"
            assert b[(k, g)] >= a[(k, g)] > 0, (a, b)
            assert a[("rocmdash_self_cpu_seconds_total:idle", g)] == 0.0  # no demoted thread on the CPU
            assert a[("rocmdash_gather_native", g)] == 0.0  # CPU: gloo host path, no RCCL
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGTERM)
        p.communicate(timeout=60)
