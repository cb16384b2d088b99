"""Query layer: reference contract of fetch_gpu_metrics (app.py:153-227), its edge
cases and behavioural parity with the reference itself."""

import math

import numpy as np
import pandas as pd
import pytest

from rocmdash.prom import query as q
from rocmdash.prom.mock import MI300_PART, FakePrometheusHTTP, SyntheticNode


def _client(node, **kw):
    return q.PrometheusClient(endpoint="http://prom:9090/api/v1/query", get=FakePrometheusHTTP(node, **kw))


def test_promql_strings_match_reference_bytes(reference_app, monkeypatch):
    # The reference builds both strings inline (app.py:157, 167-172); check ours by
    # capturing what the reference sends through a patched requests.get.
    sent = []
    node = SyntheticNode(2, host_ip="10.1.2.3")
    fake = FakePrometheusHTTP(node)

    def get(url=None, params=None, **kw):
        sent.append(params["query"])
        return fake(url=url, params=params)

    monkeypatch.setattr(reference_app.requests, "get", get)
    reference_app.fetch_gpu_metrics()
    assert sent[0] == q.node_discovery_query(reference_app.PROMETHEUS_METRICS_PODNAME)
    assert sent[1] == q.gpu_metrics_query("10.1.2.3")


def test_fetch_contract_shapes_and_dtypes():
    node = SyntheticNode(4, card_model=MI300_PART)
    df, stats = q.fetch_gpu_metrics(_client(node))
    assert list(df.index) == ["0", "1", "2", "3"] and df.index.name == "gpu_id"
    assert list(df.columns) == [
        "amd_gpu_average_package_power", "amd_gpu_edge_temperature", "amd_gpu_gfx_activity",
        "amd_gpu_total_vram", "amd_gpu_used_vram", "card_model", "vram_usage_ratio",
    ]
    assert (df["card_model"] == MI300_PART).all()
    for c in df.columns:
        if c != "card_model":
            assert df[c].dtype == np.float64
    np.testing.assert_allclose(df["vram_usage_ratio"], df["amd_gpu_used_vram"] / df["amd_gpu_total_vram"] * 100)
    assert set(stats) == {"mean", "max", "min"}
    assert "vram_usage_ratio" in stats["mean"].index and "card_model" not in stats["mean"].index


def test_parity_with_reference_on_same_data(reference_app, monkeypatch):
    node = SyntheticNode(8, seed=3)
    fake = FakePrometheusHTTP(node)
    monkeypatch.setattr(reference_app.requests, "get", fake)
    ref_df, ref_stats = reference_app.fetch_gpu_metrics()
    df, stats = q.fetch_gpu_metrics(_client(node))
    assert list(df.index) == list(ref_df.index)
    assert list(df.columns) == list(ref_df.columns)
    for c in df.columns:
        if c == "card_model":
            assert list(df[c]) == list(ref_df[c])
        else:
            np.testing.assert_allclose(df[c].astype(float), ref_df[c].astype(float))
    for k in ("mean", "max", "min"):
        pd.testing.assert_index_equal(stats[k].index, ref_stats[k].index)
        np.testing.assert_allclose(stats[k].astype(float), ref_stats[k].astype(float))


def test_lexicographic_index_like_pivot():
    node = SyntheticNode(gpu_ids=["0", "1", "10", "2"])
    df, _ = q.fetch_gpu_metrics(_client(node))
    assert list(df.index) == ["0", "1", "10", "2"]


@pytest.mark.parametrize("fault", ["duplicate", "missing_total", "http500", "no_pod", "bad_json"])
def test_error_paths_return_none_and_report(fault, reference_app, monkeypatch):
    node = SyntheticNode(2)
    kw = {}
    if fault == "duplicate":
        node.duplicate.add(("0", "amd_gpu_gfx_activity"))
    elif fault == "missing_total":
        for g in node.gpu_ids:
            node.drop.add((g, "amd_gpu_total_vram"))
    elif fault == "http500":
        kw = {"status_code": 500}
    elif fault == "no_pod":
        node.pod = "something-else"
    elif fault == "bad_json":
        kw = {"body": "<html>oops</html>"}
    errors = []
    df, stats = q.fetch_gpu_metrics(_client(node, **kw), on_error=errors.append)
    assert df is None and stats is None
    assert len(errors) == 1 and errors[0].startswith("Error fetching GPU metrics: ")
    # the reference takes the error path on the same input too
    monkeypatch.setattr(reference_app.requests, "get", FakePrometheusHTTP(node, **kw))
    assert reference_app.fetch_gpu_metrics() == (None, None)


def test_partial_metric_missing_for_one_gpu_is_nan():
    node = SyntheticNode(3)
    node.drop.add(("1", "amd_gpu_edge_temperature"))
    df, stats = q.fetch_gpu_metrics(_client(node))
    assert math.isnan(df.loc["1", "amd_gpu_edge_temperature"])
    assert not math.isnan(stats["mean"]["amd_gpu_edge_temperature"])


def test_snapshot_fast_path_equals_dataframe():
    node = SyntheticNode(8, seed=5)
    snap = q.fetch_node_snapshot(_client(node))
    df, _ = snap.to_dataframe()
    for g in snap.gpu_ids:
        for c in snap.columns:
            assert snap.value(g, c) == pytest.approx(df.loc[g, c], nan_ok=True)


def test_timeout_is_passed_to_http():
    seen = {}

    def get(url=None, params=None, timeout=None, **kw):
        seen["timeout"] = timeout
        raise RuntimeError("boom")

    c = q.PrometheusClient(endpoint="http://x", timeout=1.5, get=get)
    assert q.fetch_gpu_metrics(c, on_error=lambda m: None) == (None, None)
    assert seen["timeout"] == 1.5


def test_keepalive_client_sends_the_reference_bytes_and_reconnects():
    """The default Prometheus client (stdlib keep-alive connection) puts the SAME request
    target on the wire as requests.get(url, params={"query": q}) - the reference's call
    (app.py:158, 173) - for both reference queries; it reuses one connection, reopens a
    closed one, and raises on HTTP errors."""
    import http.server
    import threading

    import requests

    from rocmdash.prom.query import HTTPStatusError, KeepAliveGet, gpu_metrics_query, node_discovery_query

    seen = []

    class H(http.server.BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *a):
            pass

        def do_GET(self):
            seen.append((self.path, self.client_address[1]))
            code = 500 if "fail" in self.path else 200
            body = b'{"status":"success","data":{"resultType":"vector","result":[]}}'
            self.send_response(code)
            self.send_header("Content-Length", str(len(body)))
            if "close" in self.path:
                self.send_header("Connection", "close")
            self.end_headers()
            self.wfile.write(body)

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    url = f"http://127.0.0.1:{srv.server_address[1]}/api/v1/query"
    try:
        get = KeepAliveGet()
        for q in (node_discovery_query("prometheus"), gpu_metrics_query("10.0.0.7")):
            r = get(url=url, params={"query": q}, timeout=5)
            assert r.status_code == 200 and r.json()["status"] == "success"
            requests.get(url, params={"query": q}, timeout=5)
            assert seen[-2][0] == seen[-1][0], seen[-2:]  # same request target, byte for byte
        ports = [p for _, p in seen[::2]]
        assert len(set(ports)) == 1  # one keep-alive connection for both queries
        get(url=url, params={"query": "close"}, timeout=5)  # server closes: the next call reconnects
        r = get(url=url, params={"query": "up"}, timeout=5)
        assert r.status_code == 200 and seen[-1][1] != ports[0]
        with pytest.raises(HTTPStatusError):
            get(url=url, params={"query": "fail"}, timeout=5).raise_for_status()
        get.close()
        # one client shared by concurrent page sessions (Streamlit threads): every
        # thread gets its own connection, no response goes to the wrong caller
        seen.clear()
        errors = []

        def session(i):
            try:
                for k in range(20):
                    r = get(url=url, params={"query": f"s{i}_{k}"}, timeout=5)
                    assert r.status_code == 200
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        threads = [threading.Thread(target=session, args=(i,)) for i in range(4)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        assert not errors and len(seen) == 80
        by_port = {}
        for path, port in seen:
            by_port.setdefault(port, set()).add(path.rsplit("=s", 1)[1].split("_")[0])  # ...?query=s<i>_<k>
        assert len(by_port) == 4 and all(len(v) == 1 for v in by_port.values())  # one connection per thread
    finally:
        srv.shutdown()


def test_parse_text_label_cache_is_transparent():
    """parse_text caches parsed label blocks (scrapes repeat them); the cache never
    changes a result, and a bad line is still refused after its labels were cached."""
    from rocmdash.prom import exposition as ex

    text = 'a{x="1",y="q\\"z"} 1\nb{x="1",y="q\\"z"} NaN\nc 3 17\n'
    first = ex.parse_text(text)
    again = ex.parse_text(text)
    assert [tuple(s) for s in first][:1] == [tuple(s) for s in again][:1]
    assert first[0].labels == (("x", "1"), ("y", 'q"z')) and first[1].value != first[1].value
    assert first[2] == ex.Sample("c", (), 3.0, 17) and first[2].label_dict() == {}
    with pytest.raises(ValueError):
        ex.parse_text('a{x="1",y="q\\"z"} notanumber\n')
    ex._LABEL_CACHE.clear()
    assert [tuple(s)[:2] for s in ex.parse_text(text)] == [tuple(s)[:2] for s in first]
