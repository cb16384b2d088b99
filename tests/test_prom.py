"""Prometheus layer: exposition render/parse (checked against prometheus_client),
PromQL subset, the mini-Prometheus HTTP API and the exporter -> scrape -> query ->
dashboard chain over real sockets on 127.0.0.1."""

import json
import math
import urllib.request

import numpy as np
import pytest

from rocmdash.models.schema import STAT_NAMES
from rocmdash.prom import promql
from rocmdash.prom.exporter import Exporter, SyntheticSource
from rocmdash.prom.exposition import Exposition, format_value, parse_text, render_snapshot
from rocmdash.prom.mini import MiniPrometheus
from rocmdash.prom.mock import MockPrometheus, SyntheticNode
from rocmdash.prom.query import PrometheusClient, fetch_gpu_metrics, fetch_node_snapshot, gpu_metrics_query
from rocmdash.viz.panels import NodeSnapshot, build_frame


def _snap(n=3, window=True):
    cols = ("amd_gpu_edge_temperature", "amd_gpu_gfx_activity", "amd_gpu_average_package_power",
            "amd_gpu_used_vram", "amd_gpu_total_vram")
    vals = np.array([[40 + g, 10 * g, 300.5 + g, 1000 * (g + 1), 294896] for g in range(n)], float)
    w = np.random.default_rng(0).normal(size=(n, len(cols), len(STAT_NAMES))) if window else None
    return NodeSnapshot([str(g) for g in range(n)], ['102-G36236-0C "q"'] * n, cols, vals,
                        power_limits=[1400.0] * n, window=w, window_series=cols if window else ())


def test_format_value():
    assert format_value(3.0) == "3" and format_value(2.5) == "2.5"
    assert format_value(float("nan")) == "NaN" and format_value(float("inf")) == "+Inf"
    assert format_value(float("-inf")) == "-Inf" and format_value(None) == "NaN"


def test_render_parses_with_prometheus_client_and_ours():
    parser = pytest.importorskip("prometheus_client.parser")
    text = render_snapshot(_snap(), hostname="node-a")
    theirs = {}
    for fam in parser.text_string_to_metric_families(text):
        for s in fam.samples:
            theirs[(s.name, tuple(sorted(s.labels.items())))] = s.value
    ours = {(s.name, s.labels): s.value for s in parse_text(text)}
    assert theirs.keys() == ours.keys()
    for k in theirs:
        a, b = theirs[k], ours[k]
        assert (math.isnan(a) and math.isnan(b)) or a == pytest.approx(b)
    lab = dict(next(k[1] for k in ours if k[0] == "amd_gpu_gfx_activity"))
    assert lab["card_model"] == '102-G36236-0C "q"' and lab["hostname"] == "node-a"
    assert sum(1 for k in ours if k[0] == "rocmdash_window") == 3 * 5 * 6


def test_parse_escapes_and_timestamps():
    text = 'm{a="x\\"y",b="l1\\nl2",c="back\\\\slash"} 1.5 1700000000000\nm2 NaN\n# comment\n'
    s = parse_text(text)
    assert s[0].label_dict() == {"a": 'x"y', "b": "l1\nl2", "c": "back\\slash"}
    assert s[0].timestamp_ms == 1700000000000 and math.isnan(s[1].value)
    with pytest.raises(ValueError):
        parse_text("bad line with spaces {\n")


def test_exposition_help_type_once_per_family():
    e = Exposition()
    e.add("x", 1, {"a": "1"}, "help x", "counter")
    e.add("x", 2, {"a": "2"}, "help x", "counter")
    t = e.text()
    assert t.count("# TYPE x counter") == 1 and t.count("# HELP x") == 1


# ------------------------------------------------------------------------ PromQL
def test_promql_reference_queries_parse_and_match():
    sel = promql.parse('kube_pod_info{pod=~".*prometheus.*"}')
    assert sel.metric_name == "kube_pod_info"
    assert sel.matches({"__name__": "kube_pod_info", "pod": "prometheus-server-0"})
    assert not sel.matches({"__name__": "kube_pod_info", "pod": "grafana"})
    sel = promql.parse(gpu_metrics_query("10.0.0.5"))
    assert sel.matches({"__name__": "amd_gpu_gfx_activity", "instance": "10.0.0.5:5000"})
    assert not sel.matches({"__name__": "amd_gpu_gfx_activity", "instance": "10.0.0.50:5000"})  # anchored? no:
    assert not sel.matches({"__name__": "amd_gpu_gfx_activityX", "instance": "10.0.0.5:5000"})
    assert not sel.matches({"__name__": "amd_gpu_gfx_activity", "instance": "10.0.0.5"})


@pytest.mark.parametrize("q,labels,ok", [
    ('up{job="a"}', {"__name__": "up", "job": "a"}, True),
    ('up{job!="a"}', {"__name__": "up", "job": "a"}, False),
    ('up{job!~"a|b"}', {"__name__": "up", "job": "c"}, True),
    ('{__name__="up", x=""}', {"__name__": "up"}, True),
    ("up{job='single'}", {"__name__": "up", "job": "single"}, True),
    ('up{job=~"a.*",}', {"__name__": "up", "job": "abc"}, True),
])
def test_promql_matchers(q, labels, ok):
    assert promql.parse(q).matches(labels) is ok


@pytest.mark.parametrize("bad", ['{x=""}', "{}", 'up{job=~"("}', "up{job}", 'up{job="a"', "up extra", "sum(up"])
def test_promql_errors(bad):
    with pytest.raises(promql.PromQLError):
        promql.parse(bad)


def test_promql_aggregations():
    rows = [({"__name__": "m", "gpu_id": str(g % 2), "x": str(g)}, float(g)) for g in range(4)]
    e = promql.parse("sum by (gpu_id) (m)")
    got = {d["gpu_id"]: v for d, v in promql.aggregate(e, rows)}
    assert got == {"0": 2.0, "1": 4.0}
    e = promql.parse("max(m) without (x)")
    assert [v for _, v in promql.aggregate(e, rows)] == [2.0, 3.0]
    e = promql.parse("count(m)")
    assert promql.aggregate(e, rows) == [({}, 4.0)]


# -------------------------------------------------------------------- mini Prometheus
def test_tsdb_lookback_and_latest():
    p = MiniPrometheus()
    p.db.add({"__name__": "m", "a": "1"}, 1.0, ts=100.0)
    p.db.add({"__name__": "m", "a": "1"}, 2.0, ts=200.0)
    p.db.add({"__name__": "m", "a": "2"}, 5.0, ts=10.0)
    d = p.query("m", at=350.0)
    assert [(r["metric"]["a"], r["value"][1]) for r in d["result"]] == [("1", "2")]
    d = p.query("m", at=150.0)
    assert sorted((r["metric"]["a"], r["value"][1]) for r in d["result"]) == [("1", "1"), ("2", "5")]


def test_exporter_scrape_query_dashboard_end_to_end():
    """exporter (synthetic node) -> mini-Prometheus scrape over HTTP -> the
    reference's two queries over HTTP -> reference-shaped DataFrame and a frame."""
    exp = Exporter(SyntheticSource(4), hostname="node-x")
    exp.serve("127.0.0.1", 0)
    prom = MiniPrometheus(scrape_interval=0.2)
    try:
        prom.add_target(f"http://127.0.0.1:{exp.port}/metrics")
        prom.db.add({"__name__": "kube_pod_info", "pod": "prometheus-0", "host_ip": "127.0.0.1"}, 1.0)
        assert prom.scrape_all() is None
        prom.serve("127.0.0.1", 0)
        client = PrometheusClient(endpoint=f"http://127.0.0.1:{prom.port}/api/v1/query", timeout=5)
        df, stats = fetch_gpu_metrics(client, on_error=pytest.fail)
        assert list(df.index) == ["0", "1", "2", "3"]
        assert df["card_model"].iloc[0] == "102-G36236-0C"
        snap = fetch_node_snapshot(client)
        frame = build_frame(snap, snap.gpu_ids)
        assert frame.num_figures == 4 + 4 * 4
        json.loads(frame.to_json())
        with urllib.request.urlopen(f"http://127.0.0.1:{prom.port}/api/v1/targets") as r:
            t = json.load(r)["data"]["activeTargets"][0]
        assert t["health"] == "up"
        up = prom.query("up")["result"][0]
        assert up["value"][1] == "1"
        with urllib.request.urlopen(f"http://127.0.0.1:{exp.port}/metrics") as r:
            body = r.read().decode()
        assert "rocmdash_exporter_scrapes_total" in body and 'hostname="node-x"' in body
        # a bad query is a 400 with Prometheus' error envelope
        try:
            urllib.request.urlopen(f"http://127.0.0.1:{prom.port}/api/v1/query?query=%7B%7D")
            raise AssertionError("expected HTTP 400")
        except urllib.error.HTTPError as e:
            assert e.code == 400 and json.load(e)["status"] == "error"
    finally:
        prom.close()
        exp.close()


def test_down_target_sets_up_zero():
    prom = MiniPrometheus(timeout=0.5)
    t = prom.add_target("http://127.0.0.1:9/metrics")
    assert prom.scrape_once(t) is False
    assert prom.query("up")["result"][0]["value"][1] == "0" and t.health == "down"


def test_mock_prometheus_http_serves_reference_queries():
    mp = MockPrometheus(SyntheticNode(8))
    mp.serve("127.0.0.1", 0)
    try:
        client = PrometheusClient(endpoint=f"http://127.0.0.1:{mp.port}/api/v1/query")
        df, _ = fetch_gpu_metrics(client, on_error=pytest.fail)
        assert len(df) == 8
    finally:
        mp.close()


def test_histogram_exposition_parses_with_prometheus_client():
    parser = pytest.importorskip("prometheus_client.parser")
    from rocmdash.utils.timing import LatencyHistogram

    h = LatencyHistogram("rocmdash_test_seconds", "test")
    for v in (1e-6, 3e-4, 0.002, 0.002, 7.0):
        h.observe(v)
    e = Exposition()
    h.add_to(e, {"gpu_id": "0"})
    fams = list(parser.text_string_to_metric_families(e.text()))
    assert len(fams) == 1 and fams[0].type == "histogram" and fams[0].name == "rocmdash_test_seconds"
    samples = {(s.name, s.labels.get("le")): s.value for s in fams[0].samples}
    assert samples[("rocmdash_test_seconds_count", None)] == 5
    assert samples[("rocmdash_test_seconds_bucket", "+Inf")] == 5
    assert samples[("rocmdash_test_seconds_bucket", "0.0025")] == 4
    assert samples[("rocmdash_test_seconds_bucket", "1e-05")] == 1


def test_percentile_matches_numpy():
    from rocmdash.utils.timing import Stopwatch, percentile

    v = sorted(np.random.default_rng(0).normal(size=101).tolist())
    for q in (0, 10, 50, 90, 99, 100):
        assert percentile(v, q) == pytest.approx(np.percentile(v, q))
    sw = Stopwatch()
    for _ in range(3):
        with sw.lap():
            pass
    assert sw.summary()["n"] == 3


def test_healthz_follows_the_refresh_loop():
    """/healthz is 200 while the node service keeps refreshing and 503 once it stalls
    (the DaemonSet's liveness probe then restarts the container)."""
    import time

    from rocmdash.serve import _Latest

    latest = _Latest(stall_s=0.3)
    exp = Exporter(latest)
    exp.serve("127.0.0.1", 0)

    def code():
        try:
            with urllib.request.urlopen(f"http://127.0.0.1:{exp.port}/healthz") as r:
                return r.status, r.read().decode()
        except urllib.error.HTTPError as e:
            return e.code, e.read().decode()

    try:
        assert code()[0] == 200  # starting up: within the stall budget
        latest.set(_snap(2), None)
        c, body = code()
        assert c == 200 and "last refresh" in body
        time.sleep(0.4)
        c, body = code()
        assert c == 503 and "last refresh" in body
        latest.set(_snap(2), None)
        assert code()[0] == 200
        assert Exporter(SyntheticSource(1)).health() == (True, "OK")
    finally:
        exp.close()


def test_node_window_exposition_and_page_table():
    """Node-wide window statistics travel in the snapshot: one rocmdash_node_window
    family with metric/stat labels (no gpu_id), and the page's table form."""
    from rocmdash.models.schema import NUM_STATS
    from rocmdash.prom.exposition import parse_text, render_snapshot
    from rocmdash.ui.page import node_window_table
    from rocmdash.viz.panels import NodeSnapshot

    series = ("amd_gpu_edge_temperature", "amd_gpu_average_package_power")
    nw = np.arange(len(series) * NUM_STATS, dtype=np.float64).reshape(len(series), NUM_STATS)
    snap = NodeSnapshot(gpu_ids=["0", "1"], card_models=["102-G36236-0C"] * 2, columns=series,
                        values=[[40.0, 500.0], [41.0, 520.0]], window=np.zeros((2, 2, NUM_STATS)),
                        window_series=series, node_window=nw)
    samples = [s for s in parse_text(render_snapshot(snap, hostname="n1")) if s.name == "rocmdash_node_window"]
    got = {(s.label_dict()["metric"], s.label_dict()["stat"]): s.value for s in samples}
    assert got[("amd_gpu_average_package_power", "p99")] == nw[1, 5] and got[("amd_gpu_edge_temperature", "count")] == 7
    assert all("gpu_id" not in s.label_dict() for s in samples)
    table = node_window_table(snap)
    assert table["amd_gpu_edge_temperature"]["max"] == 1.0 and "last" not in table["amd_gpu_edge_temperature"]


def test_xcd_exposition_and_page_table():
    """Per-XCD busy / clocks travel in the snapshot: amd_gpu_xcd_activity and
    amd_gpu_xcd_gfx_clock per (gpu_id, xcd); XCDs the firmware reports none for (NaN)
    are left out; the page's table covers the selected GPUs only."""
    from rocmdash.prom.exposition import parse_text, render_snapshot
    from rocmdash.ui.page import xcd_table
    from rocmdash.viz.panels import NodeSnapshot

    xcd = np.full((2, 2, 8), np.nan, dtype=np.float32)
    xcd[0, 0], xcd[0, 1] = np.arange(8) * 10, 2400 - np.arange(8)
    xcd[1, 0, :4], xcd[1, 1, :4] = 50.0, 2000.0  # e.g. a part/mode with four XCDs
    snap = NodeSnapshot(gpu_ids=["0", "1"], card_models=["102-G36236-0C"] * 2, columns=("amd_gpu_gfx_activity",),
                        values=[[30.0], [50.0]], xcd=xcd)
    samples = parse_text(render_snapshot(snap))
    act = {(s.label_dict()["gpu_id"], s.label_dict()["xcd"]): s.value for s in samples if s.name == "amd_gpu_xcd_activity"}
    clk = {(s.label_dict()["gpu_id"], s.label_dict()["xcd"]): s.value for s in samples if s.name == "amd_gpu_xcd_gfx_clock"}
    assert len(act) == len(clk) == 12
    assert act[("0", "7")] == 70.0 and clk[("0", "3")] == 2397.0 and act[("1", "3")] == 50.0
    assert ("1", "4") not in act
    table = xcd_table(snap, ["1"])
    assert list(table) == ["GPU 1"] and table["GPU 1"]["XCD 0 MHz"] == 2000.0 and "XCD 4 busy %" not in table["GPU 1"]
    assert xcd_table(NodeSnapshot(gpu_ids=["0"], card_models=[""], columns=(), values=[[]])) is None


def test_board_identity_and_refresh_time_round_trip():
    """A part number the SKU table does not know still resolves through the exported
    amd-smi product name (``amd_gpu_info``), and the node refresh time travels with the
    extended query: Prometheus mode names the board like native mode does."""
    from rocmdash.prom.snapshot_io import extended_query, merge_extended, snapshot_from_series

    snap = _snap(2)
    snap.card_models = ["102-G99999-0C"] * 2  # not in GPU_NAME_RESOLVE
    snap.product_names = ["AMD Instinct MI355 OAM", "AMD Instinct MI355 OAM"]
    text = render_snapshot(snap) + "rocmdash_node_refresh_timestamp_seconds 1700000000.25\n"
    items = [(dict(s.labels, __name__=s.name), s.value) for s in parse_text(text)]
    info = [lab for lab, _ in items if lab["__name__"] == "amd_gpu_info"]
    assert len(info) == 2 and info[0]["product_name"] == "AMD Instinct MI355 OAM"
    assert "amd_gpu_info" in extended_query("10.0.0.1") and "rocmdash_node_refresh_timestamp_seconds" in extended_query("x")
    direct = snapshot_from_series(items)
    assert direct.refresh_time == 1700000000.25 and direct.model_name(0) == "MI355X"
    compat = NodeSnapshot(["0", "1"], ["102-G99999-0C"] * 2, snap.columns, snap.values)
    assert compat.model_name(0) is None  # the reference's lookup alone: "(None)"
    merged = merge_extended(compat, snapshot_from_series(items, require_vram=False))
    assert merged.model_name(1) == "MI355X" and merged.refresh_time == 1700000000.25


def test_mini_prometheus_json_fast_path_matches_the_dict_path():
    """The HTTP handler's query_json (cached label JSON and result elements) answers
    exactly what json.dumps of query() does, before and after new samples arrive, for
    selectors with regex name and label matchers (the page's queries)."""
    import json

    from rocmdash.prom.mini import MiniPrometheus

    prom = MiniPrometheus()
    for g in range(3):
        for name in ("amd_gpu_gfx_activity", "amd_gpu_used_vram", "rocmdash_window"):
            prom.db.add({"__name__": name, "gpu_id": str(g), "instance": f"10.0.0.{g % 2}:9400"}, g * 1.5, ts=100.0)
    qs = ['{__name__=~"amd_gpu_gfx_activity|rocmdash_window", instance=~"10.0.0.1:.+"}', "amd_gpu_used_vram",
          'amd_gpu_gfx_activity{gpu_id!="1"}']
    for at in (101.0, 102.0):
        for q in qs:
            prom.query(q, at)  # parse + cache
            assert json.loads(prom.query_json(q, at)) == {"status": "success", "data": prom.query(q, at)}, q
        prom.db.add({"__name__": "amd_gpu_gfx_activity", "gpu_id": "1", "instance": "10.0.0.1:9400"}, 7.25, ts=101.5)
    got = json.loads(prom.query_json(qs[0], 102.0))["data"]["result"]
    assert {"gpu_id": "1", "instance": "10.0.0.1:9400", "__name__": "amd_gpu_gfx_activity"} in [r["metric"] for r in got]
    assert ["101.5" in json.dumps(r["value"]) for r in got].count(True) == 1


def test_mini_prometheus_parses_each_query_once_beyond_the_cache_size(monkeypatch):
    """query_json parses and evaluates once per request, also past 256 distinct
    queries (bounded LRU), and bad PromQL raises PromQLError directly."""
    import pytest

    from rocmdash.prom import mini
    from rocmdash.prom.promql import PromQLError

    prom = mini.MiniPrometheus()
    prom.db.add({"__name__": "amd_gpu_gfx_activity", "gpu_id": "0"}, 5.0)
    calls = []
    real = mini.parse
    monkeypatch.setattr(mini, "parse", lambda q: calls.append(q) or real(q))
    for i in range(300):
        prom.query_json(f'amd_gpu_gfx_activity{{gpu_id="{i % 300}"}}')
    assert len(calls) == 300 and prom.queries == 300 and len(prom._parsed) == 256
    q = 'amd_gpu_gfx_activity{gpu_id="0"}'
    calls.clear()
    prom.query_json(q)  # evicted long ago: parsed again, once
    prom.query_json(q)  # cached now
    assert calls == [q] and prom.queries == 302
    with pytest.raises(PromQLError):
        prom.query_json("sum(")
