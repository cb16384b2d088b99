"""The Streamlit page driven through the recording Streamlit double, side by side with
the reference app.py on the same synthetic Prometheus data: same call sequence,
same figures (JSON-equal), same headers, statistics and widget keys."""

import importlib.util
import json
import os

import numpy as np
import pytest

from rocmdash.prom import query as q
from rocmdash.prom.mock import MI300_PART, FakePrometheusHTTP, SyntheticNode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Stop(Exception):
    pass


def _import_our_app():
    spec = importlib.util.spec_from_file_location("rocmdash_app", os.path.join(ROOT, "app.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _run_reference(reference_app, st, node, monkeypatch, widget_values=None):
    monkeypatch.setattr(reference_app.requests, "get", FakePrometheusHTTP(node))

    def stop(_):
        raise _Stop()

    monkeypatch.setattr(reference_app.time, "sleep", stop)
    st.reset()
    st.WIDGET_VALUES.update(widget_values or {})
    with pytest.raises(_Stop):
        reference_app.main()
    return list(st.CALLS)


def _run_ours(st, node, monkeypatch, widget_values=None):
    app = _import_our_app()
    fake = FakePrometheusHTTP(node)
    monkeypatch.setattr(q.PrometheusClient, "_http_get", lambda self: fake)
    st.reset()
    st.WIDGET_VALUES.update(widget_values or {})
    app.main(max_refreshes=1, data_source="prometheus")
    return list(st.CALLS)


def _fig_json(x):
    if hasattr(x, "to_json"):
        return json.loads(x.to_json())
    return json.loads(json.dumps(x))


def _compare(ref_calls, our_calls):
    def kinds(calls):
        return [c[0] for c in calls if c[0] not in ("enter",)]

    assert kinds(our_calls) == kinds(ref_calls)
    ref_figs = [c for c in ref_calls if c[0] == "plotly_chart"]
    our_figs = [c for c in our_calls if c[0] == "plotly_chart"]
    assert len(ref_figs) == len(our_figs)
    for r, o in zip(ref_figs, our_figs):
        assert _fig_json(o[1][0]) == _fig_json(r[1][0])
        assert o[2]["key"].rsplit("_", 1)[0] == r[2]["key"].rsplit("_", 1)[0]  # same key minus timestamp
    for name in ("title", "markdown", "header", "subheader", "checkbox", "toggle", "sidebar.write"):
        rc = [(c[1], {k: v for k, v in c[2].items()}) for c in ref_calls if c[0] == name]
        oc = [(c[1], {k: v for k, v in c[2].items()}) for c in our_calls if c[0] == name]
        assert oc == rc, name
    rd = [c for c in ref_calls if c[0] == "dataframe"]
    od = [c for c in our_calls if c[0] == "dataframe"]
    assert len(rd) == len(od) == 1
    rdf, odf = rd[0][1][0], od[0][1][0]
    assert sorted(rdf.index) == sorted(odf.index) and list(rdf.columns) == list(odf.columns)
    # The reference's .round(2) is a no-op on its object-dtype stats (app.py:480); ours
    # rounds as intended, so compare to half a cent.
    np.testing.assert_allclose(odf.loc[rdf.index].to_numpy(float), rdf.to_numpy(float), rtol=0, atol=0.005 + 1e-9)
    rt = [c for c in ref_calls if c[0] == "text"][-1][1][0]
    ot = [c for c in our_calls if c[0] == "text"][-1][1][0]
    assert rt[:14] == ot[:14] == "Last updated: "


@pytest.mark.parametrize("select_all,gauge", [(False, True), (True, True), (True, False)])
def test_page_matches_reference(reference_app, st_stub, monkeypatch, select_all, gauge):
    node = SyntheticNode(8, card_model=MI300_PART, seed=11)
    node.overrides[("3", "amd_gpu_average_package_power")] = 0  # idle GPU: excluded from power mean
    widgets = {"Use Gauge Visualization": gauge}
    if select_all:
        widgets.update({f"gpu_checkbox_{g}": True for g in range(8)})
    ref = _run_reference(reference_app, st_stub, node, monkeypatch, widgets)
    ours = _run_ours(st_stub, node, monkeypatch, widgets)
    _compare(ref, ours)
    n_sel = 8 if select_all else 1
    assert len([c for c in ours if c[0] == "plotly_chart"]) == 4 + 4 * n_sel


def test_page_unknown_model_header_and_power_axis(st_stub, monkeypatch):
    node = SyntheticNode(2, card_model="999-UNKNOWN")
    calls = _run_ours(st_stub, node, monkeypatch)
    headers = [c[1][0] for c in calls if c[0] == "markdown" and str(c[1][0]).startswith("###")]
    assert headers == ["### GPU 0 (None)"]
    power = [c for c in calls if c[0] == "plotly_chart" and c[2]["key"].startswith("plot_power_0")][0]
    assert power[1][0]["data"][0]["gauge"]["axis"]["range"] == [0, 300]


def test_page_mi355x_model_resolves(st_stub, monkeypatch):
    node = SyntheticNode(1)  # MI355X part number
    calls = _run_ours(st_stub, node, monkeypatch)
    headers = [c[1][0] for c in calls if c[0] == "markdown" and str(c[1][0]).startswith("###")]
    assert headers == ["### GPU 0 (MI355X)"]
    power = [c for c in calls if c[0] == "plotly_chart" and c[2]["key"].startswith("plot_power_0")][0]
    assert power[1][0]["data"][0]["gauge"]["axis"]["range"] == [0, 1400]


def test_page_prometheus_down_shows_error_and_empty_selection(st_stub, monkeypatch):
    app = _import_our_app()
    fake = FakePrometheusHTTP(SyntheticNode(2), status_code=503)
    monkeypatch.setattr(q.PrometheusClient, "_http_get", lambda self: fake)
    st_stub.reset()
    app.main(max_refreshes=1, data_source="prometheus")
    errs = st_stub.calls("error")
    assert len(errs) == 2 and errs[0][1][0].startswith("Error fetching GPU metrics")
    assert not st_stub.calls("checkbox") and not st_stub.calls("plotly_chart")


def test_page_synthetic_source_and_natural_sort(st_stub, monkeypatch):
    app = _import_our_app()
    monkeypatch.setenv("ROCMDASH_SYNTHETIC_GPUS", "12")
    from rocmdash.ui import page

    page._DataSource._synthetic = None
    st_stub.reset()
    app.main(max_refreshes=1, data_source="synthetic")
    labels = [c[1][0] for c in st_stub.calls("checkbox")]
    assert labels == [f"GPU {i}" for i in range(12)]  # natural order: 2 before 10
    page._DataSource._synthetic = None


def test_app_module_level_api(st_stub):
    app = _import_our_app()
    for name in ("PROMETHEUS_METRICS_ENDPOINT", "PROMETHEUS_METRICS_PODNAME", "REFRESH_INTERVAL", "GPU_NAME_RESOLVE",
                 "GPU_POWER_LIMITS", "GAUGE_COLORS", "get_color_for_value", "create_gauge", "create_horizontal_bar",
                 "fetch_gpu_metrics", "get_power_limit", "create_visualization", "main"):
        assert hasattr(app, name), name
    assert st_stub.CALLS[0][0] == "set_page_config"
    assert st_stub.CALLS[0][2]["page_title"] == "GPU Metrics Dashboard"
    assert app.get_power_limit("102-G30211-0C") == 750 and app.get_power_limit("nope") == 300
    assert app.PROMETHEUS_METRICS_ENDPOINT == "http://localhost:9090/api/v1/query"
