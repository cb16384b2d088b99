"""Colour bands and figure factories: semantics of app.py:56-151, JSON parity with
Plotly (our figures serialise to the same tree as the reference's go.Figure)."""

import json
import math

import numpy as np
import pytest

from rocmdash.viz.figures import (
    GAUGE_COLORS,
    Figure,
    create_chart,
    create_gauge,
    create_horizontal_bar,
    get_color_for_value,
)


@pytest.mark.parametrize(
    "value,expected",
    [
        (0, "green"), (20, "green"), (20.0001, "light_green"), (40, "light_green"), (40.5, "yellow"),
        (60, "yellow"), (61, "orange"), (80, "orange"), (80.01, "red"), (100, "red"), (150, "red"),
        (-5, "green"),
    ],
)
def test_color_bands_inclusive_upper_bounds(value, expected):
    assert get_color_for_value(value, 100) == GAUGE_COLORS[expected]


def test_color_band_edge_cases():
    with pytest.raises(ZeroDivisionError):
        get_color_for_value(10, 0)
    assert get_color_for_value(float("nan"), 100) == GAUGE_COLORS["red"]
    assert get_color_for_value(300, 1400) == GAUGE_COLORS["light_green"]  # 21.4 %


def _plotly_gauge(value, title, min_val=0, max_val=100, height=400):
    go = pytest.importorskip("plotly.graph_objects")
    color = get_color_for_value(value, max_val)
    fig = go.Figure(go.Indicator(
        mode="gauge+number", value=value, title={"text": title},
        gauge={
            "axis": {"range": [min_val, max_val], "tickmode": "linear", "tick0": min_val, "dtick": max_val / 5,
                     "showticklabels": True},
            "bar": {"color": color, "line": {"color": "black", "width": 1}},
            "steps": [
                {"range": [0, max_val * 0.2], "color": GAUGE_COLORS["plate_green"]},
                {"range": [max_val * 0.2, max_val * 0.4], "color": GAUGE_COLORS["plate_light_green"]},
                {"range": [max_val * 0.4, max_val * 0.6], "color": GAUGE_COLORS["plate_yellow"]},
                {"range": [max_val * 0.6, max_val * 0.8], "color": GAUGE_COLORS["plate_orange"]},
                {"range": [max_val * 0.8, max_val], "color": GAUGE_COLORS["plate_red"]},
            ],
        },
    ))
    fig.update_layout(height=height, margin=dict(l=30, r=30, t=0, b=0))
    return fig


def _plotly_bar(value, title, min_val=0, max_val=100, height=400):
    go = pytest.importorskip("plotly.graph_objects")
    color = get_color_for_value(value, max_val)
    fig = go.Figure(go.Bar(x=[value], y=[title], orientation="h", marker_color=color, marker_line_color="gray",
                           marker_line_width=2, width=0.5))
    fig.update_layout(xaxis=dict(range=[min_val, max_val], showgrid=True, gridcolor="lightgray"),
                      yaxis=dict(showticklabels=False), height=height, margin=dict(l=20, r=20, t=20, b=20),
                      showlegend=False)
    for start, end, c in [
        (0, max_val * 0.2, GAUGE_COLORS["plate_green"]),
        (max_val * 0.2, max_val * 0.4, GAUGE_COLORS["plate_light_green"]),
        (max_val * 0.4, max_val * 0.6, GAUGE_COLORS["plate_yellow"]),
        (max_val * 0.6, max_val * 0.8, GAUGE_COLORS["plate_orange"]),
        (max_val * 0.8, max_val, GAUGE_COLORS["plate_red"]),
    ]:
        fig.add_shape(type="rect", x0=start, x1=end, y0=-0.5, y1=0.5, fillcolor=c, opacity=0.3, layer="below",
                      line_width=0)
    return fig


CASES = [
    (42.5, "Avg GPU Utilization (%)", 100, 300),
    (0, "Temperature (°C)", 100, 200),
    (812.0, "Power Usage (W)", 1400, 200),
    (np.float64(99.99), "VRAM Usage (%)", 100, 200),
    (151, "Avg Power Usage (W)", 300, 300),
    (7, "x", 750, 400),
]


@pytest.mark.parametrize("value,title,max_val,height", CASES)
def test_gauge_json_matches_plotly(value, title, max_val, height):
    ours = json.loads(create_gauge(value, title, max_val=max_val, height=height).to_json())
    ref = json.loads(_plotly_gauge(value, title, max_val=max_val, height=height).to_json())
    assert ours == ref


@pytest.mark.parametrize("value,title,max_val,height", CASES)
def test_bar_json_matches_plotly(value, title, max_val, height):
    ours = json.loads(create_horizontal_bar(value, title, max_val=max_val, height=height).to_json())
    ref = json.loads(_plotly_bar(value, title, max_val=max_val, height=height).to_json())
    assert ours == ref


def test_nan_value_serialises_as_null_like_plotly():
    ours = json.loads(create_gauge(float("nan"), "t").to_json())
    ref = json.loads(_plotly_gauge(float("nan"), "t").to_json())
    assert ours == ref
    assert ours["data"][0]["value"] is None


def test_to_plotly_roundtrip_and_dict():
    go = pytest.importorskip("plotly.graph_objects")
    fig = create_gauge(33, "t", max_val=300, height=250)
    pf = fig.to_plotly()
    assert isinstance(pf, go.Figure)
    assert json.loads(pf.to_json()) == json.loads(fig.to_json())
    d = fig.to_dict()
    assert d["layout"]["height"] == 250 and "template" in d["layout"]


def test_figure_update_layout_and_add_shape_magic_underscores():
    f = Figure([{"type": "bar", "x": [1]}], {})
    f.update_layout(margin=dict(l=1), height=10, title_text="hello")
    f.add_shape(type="line", x0=0, x1=1, line_width=3, line_color="red")
    assert f.layout["margin"] == {"l": 1}
    assert f.layout["title"] == {"text": "hello"}
    assert f.layout["shapes"][0]["line"] == {"width": 3, "color": "red"}
    json.loads(f.to_json())


def test_create_chart_dispatch():
    assert create_chart(1, "a", 100, 10, True).data[0]["type"] == "indicator"
    assert create_chart(1, "a", 100, 10, False).data[0]["type"] == "bar"


def test_fast_path_is_faster_than_plotly():
    import time

    pytest.importorskip("plotly")
    t0 = time.perf_counter()
    for i in range(20):
        _plotly_gauge(float(i), "t").to_json()
    t_ref = time.perf_counter() - t0
    t0 = time.perf_counter()
    for i in range(20):
        create_gauge(float(i), "t").to_json()
    t_ours = time.perf_counter() - t0
    assert t_ours * 5 < t_ref, (t_ours, t_ref)
    assert not math.isnan(t_ours)
