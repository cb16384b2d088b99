"""Gauge / bar figure factories that emit Plotly-compatible figure JSON without Plotly.

Reference: ``create_gauge`` (``app.py:70-103``), ``create_horizontal_bar``
(``app.py:105-151``) and ``get_color_for_value`` (``app.py:56-68``). The reference
builds a validated ``plotly.graph_objects.Figure`` per chart and Streamlit then
serialises it; at 8 GPUs that is 36 figures and ~150 ms per refresh on a CPU
(BASELINE.md), i.e. the whole dashboard refresh is Plotly object construction.

Here a figure is a plain ``{"data": [...], "layout": {...}}`` tree built from dict
literals (no validation pass: the trees are fixed by construction and the test suite
checks them against Plotly's own JSON, ``tests/test_viz.py``). The default Plotly
template (~7 KB of JSON, identical for every figure) is serialised ONCE per process
and spliced into each figure's JSON, so a refresh costs a few microseconds per chart.
``Figure.to_plotly()`` gives a real ``go.Figure`` when a consumer needs one.
"""

from __future__ import annotations

import json
import math
from functools import lru_cache

# Colour scheme, verbatim from app.py:41-54.
GAUGE_COLORS = {
    "green": "#2ecc71",  # 0-20% (value bar)
    "light_green": "#27ae60",  # 20-40% (value bar)
    "yellow": "#f1c40f",  # 40-60% (value bar)
    "orange": "#e67e22",  # 60-80% (value bar)
    "red": "#e74c3c",  # 80-100% (value bar)
    # Less saturated colours for gauge plates
    "plate_green": "#a8e6cf",
    "plate_light_green": "#88d8b0",
    "plate_yellow": "#ffd3b6",
    "plate_orange": "#ffaaa5",
    "plate_red": "#ff8b94",
}

_PLATES = ("plate_green", "plate_light_green", "plate_yellow", "plate_orange", "plate_red")


def get_color_for_value(value, max_val):
    """Bar colour by percentage of ``max_val`` (app.py:56-68).

    Same semantics as the reference: inclusive upper bounds at 20/40/60/80 %,
    ``max_val == 0`` raises ``ZeroDivisionError``, NaN falls through to red.
    """
    percentage = (value / max_val) * 100
    if percentage <= 20:
        return GAUGE_COLORS["green"]
    elif percentage <= 40:
        return GAUGE_COLORS["light_green"]
    elif percentage <= 60:
        return GAUGE_COLORS["yellow"]
    elif percentage <= 80:
        return GAUGE_COLORS["orange"]
    return GAUGE_COLORS["red"]


# ----------------------------------------------------------------------------- JSON
def _num(x):
    """Plotly's JSON encoder semantics for a scalar: numpy scalars -> Python numbers,
    NaN / inf -> null; ints stay ints."""
    if x is None:
        return None
    if isinstance(x, bool):
        return x
    if isinstance(x, int):
        return x
    try:
        f = float(x)
    except (TypeError, ValueError):
        return x
    if math.isnan(f) or math.isinf(f):
        return None
    if hasattr(x, "dtype") and getattr(x.dtype, "kind", "f") in "iu":
        return int(x)
    return f


@lru_cache(maxsize=1)
def template_json() -> str:
    """The default Plotly template as JSON (what ``go.Figure().to_json()`` embeds).

    Taken from the installed Plotly when present; without Plotly the layout carries an
    empty template (Plotly.js then uses its own defaults)."""
    try:
        import plotly.io as pio

        name = pio.templates.default
        if not name or name == "none":
            return "{}"
        return json.dumps(pio.templates[name].to_plotly_json(), separators=(",", ":"))
    except Exception:
        return "{}"


def _dumps(obj) -> str:
    return json.dumps(obj, separators=(",", ":"), allow_nan=False)


def _set_path(d: dict, key: str, value) -> None:
    """Plotly 'magic underscore' keys: line_width -> {'line': {'width': ...}}."""
    parts = key.split("_") if key not in _NO_SPLIT else [key]
    cur = d
    for p in parts[:-1]:
        nxt = cur.get(p)
        if not isinstance(nxt, dict):
            nxt = {}
            cur[p] = nxt
        cur = nxt
    cur[parts[-1]] = value


# property names that contain underscores and must not be split
_NO_SPLIT = frozenset({"use_container_width"})


def _merge(dst: dict, src: dict) -> None:
    for k, v in src.items():
        if "_" in k and k not in dst and k not in _NO_SPLIT and k.split("_")[0] in _MAGIC_ROOTS:
            _set_path(dst, k, _clean(v))
        elif isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = _clean(v)


_MAGIC_ROOTS = frozenset({"line", "marker", "title", "xaxis", "yaxis", "font", "legend", "margin"})


def _clean(v):
    if isinstance(v, dict):
        return {k: _clean(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_clean(x) for x in v]
    if isinstance(v, str):
        return v
    return _num(v)


class Figure:
    """Minimal Plotly-figure stand-in: ``data``/``layout`` trees plus the methods the
    reference's factories call (``update_layout``, ``add_shape``) and serialisation.

    ``to_json()`` / ``to_dict()`` are structurally identical to Plotly's for the
    figures this module builds (checked in tests/test_viz.py).

    Figures made by the factories below are *lazy*: they keep (kind, value, title,
    axis range, height) and serialise through a cached JSON template of that panel
    (only the value and the band colour change between refreshes), so a gauge costs a
    few string concatenations per refresh. The ``data`` / ``layout`` trees are built
    only when accessed; any mutation switches the figure to the tree path.
    """

    __slots__ = ("_data", "_layout", "_fast")

    def __init__(self, data=None, layout=None, _fast=None):
        self._fast = _fast
        if _fast is None:
            self._data = list(data or [])
            self._layout = dict(layout or {})
        else:
            self._data = None
            self._layout = None

    def _materialize(self):
        if self._data is None:
            kind, value, title, min_val, max_val, height = self._fast
            d, lay = _BUILDERS[kind](value, title, min_val, max_val, height)
            self._data, self._layout = d, lay

    @property
    def data(self):
        self._materialize()
        self._fast = None  # the caller may mutate the tree
        return self._data

    @data.setter
    def data(self, v):
        self._materialize()
        self._fast = None
        self._data = list(v)

    @property
    def layout(self):
        self._materialize()
        self._fast = None  # the caller may mutate the tree
        return self._layout

    @layout.setter
    def layout(self, v):
        self._materialize()
        self._fast = None
        self._layout = dict(v)

    def update_layout(self, dict1=None, **kwargs):
        lay = self.layout
        if dict1:
            _merge(lay, dict1)
        if kwargs:
            _merge(lay, kwargs)
        return self

    def add_shape(self, **kwargs):
        shape = {}
        for k, v in kwargs.items():
            if "_" in k:
                _set_path(shape, k, _clean(v))
            else:
                shape[k] = _clean(v)
        self.layout.setdefault("shapes", []).append(shape)
        return self

    def to_dict(self) -> dict:
        self._materialize()
        layout = {"template": json.loads(template_json())}
        layout.update(self._layout)
        return {"data": self._data, "layout": layout}

    to_plotly_json = to_dict

    def json_parts(self) -> tuple:
        """The figure's JSON as a few strings to concatenate (no copy of the ~7 KB
        template per figure when a caller joins many figures)."""
        if self._fast is not None:
            kind, value, title, min_val, max_val, height = self._fast
            head, mid, tail = _json_template(kind, title, min_val, max_val, height)
            return head, get_color_for_value(value, max_val), mid, _value_json(value), tail
        return (self.to_json(),)

    def to_json(self) -> str:
        if self._fast is not None:
            return "".join(self.json_parts())
        body = _dumps(self._layout)
        tmpl = template_json()
        layout = '{"template":' + tmpl + ("," + body[1:] if len(body) > 2 else "}")
        return '{"data":' + _dumps(self._data) + ',"layout":' + layout + "}"

    def to_plotly(self):
        """A real ``plotly.graph_objects.Figure`` (requires Plotly)."""
        import plotly.graph_objects as go

        return go.Figure(self.to_dict())

    def __repr__(self) -> str:
        self._materialize()
        kinds = ",".join(t.get("type", "?") for t in self._data)
        return f"Figure(data=[{kinds}], layout_keys={sorted(self._layout)})"


_INF = float("inf")
_NINF = float("-inf")
_COLOR_MARK = "@@ROCMDASH_COLOR@@"
_VALUE_MARK = "@@ROCMDASH_VALUE@@"


def _value_json(value) -> str:
    if type(value) is float:  # the common case: a finite Python float
        if value == value and value not in (_INF, _NINF):
            return repr(value)
        return "null"
    v = _num(value)
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return repr(v)
    return json.dumps(v)


@lru_cache(maxsize=4096)
def _json_template(kind, title, min_val, max_val, height):
    """(head, mid, tail) such that head + colour + mid + value + tail is the figure's
    JSON (the colour precedes the value in both trace layouts)."""
    d, lay = _BUILDERS[kind](_VALUE_MARK, title, min_val, max_val, height, color=_COLOR_MARK)
    text = Figure(d, lay).to_json()
    c = text.index(json.dumps(_COLOR_MARK))
    v = text.index(json.dumps(_VALUE_MARK))
    assert c < v and text.count(_COLOR_MARK) == 1 and text.count(_VALUE_MARK) == 1
    return (text[:c] + '"', '"' + text[c + len(json.dumps(_COLOR_MARK)) : v], text[v + len(json.dumps(_VALUE_MARK)) :])


# ------------------------------------------------------------------------ factories
@lru_cache(maxsize=256)
def _gauge_steps(max_val):
    return tuple(
        (max_val * lo if lo else 0, max_val * hi if hi < 1.0 else max_val, GAUGE_COLORS[p])
        for (lo, hi), p in zip(((0, 0.2), (0.2, 0.4), (0.4, 0.6), (0.6, 0.8), (0.8, 1.0)), _PLATES)
    )


def _gauge_tree(value, title, min_val, max_val, height, color=None):
    color = get_color_for_value(value, max_val) if color is None else color
    steps = [{"color": c, "range": [_num(lo), _num(hi)]} for lo, hi, c in _gauge_steps(max_val)]
    trace = {
        "gauge": {
            "axis": {
                "dtick": _num(max_val / 5),
                "range": [_num(min_val), _num(max_val)],
                "showticklabels": True,
                "tick0": _num(min_val),
                "tickmode": "linear",
            },
            "bar": {"color": color, "line": {"color": "black", "width": 1}},
            "steps": steps,
        },
        "mode": "gauge+number",
        "title": {"text": title},
        "value": value if value is _VALUE_MARK else _num(value),
        "type": "indicator",
    }
    return [trace], {"margin": {"l": 30, "r": 30, "t": 0, "b": 0}, "height": _num(height)}


def _bar_tree(value, title, min_val, max_val, height, color=None):
    color = get_color_for_value(value, max_val) if color is None else color
    trace = {
        "marker": {"color": color, "line": {"color": "gray", "width": 2}},
        "orientation": "h",
        "width": 0.5,
        "x": [value if value is _VALUE_MARK else _num(value)],
        "y": [title],
        "type": "bar",
    }
    shapes = [
        {
            "fillcolor": c,
            "layer": "below",
            "line": {"width": 0},
            "opacity": 0.3,
            "type": "rect",
            "x0": _num(lo),
            "x1": _num(hi),
            "y0": -0.5,
            "y1": 0.5,
        }
        for lo, hi, c in _gauge_steps(max_val)
    ]
    layout = {
        "xaxis": {"range": [_num(min_val), _num(max_val)], "showgrid": True, "gridcolor": "lightgray"},
        "yaxis": {"showticklabels": False},
        "margin": {"l": 20, "r": 20, "t": 20, "b": 20},
        "height": _num(height),
        "showlegend": False,
        "shapes": shapes,
    }
    return [trace], layout


_BUILDERS = {"gauge": _gauge_tree, "bar": _bar_tree}


def _hashable(x) -> bool:
    try:
        hash(x)
        return True
    except TypeError:
        return False


def _make(kind, value, title, min_val, max_val, height) -> Figure:
    get_color_for_value(value, max_val)  # reference semantics: max_val == 0 raises here
    if isinstance(title, str) and _hashable(min_val) and _hashable(max_val) and _hashable(height):
        return Figure(_fast=(kind, value, title, min_val, max_val, height))
    d, lay = _BUILDERS[kind](value, title, min_val, max_val, height)
    return Figure(d, lay)


def create_gauge(value, title, min_val=0, max_val=100, height=400) -> Figure:
    """Gauge chart (app.py:70-103): 5 pastel plate steps at 20 % bands, value bar in
    the band colour with a 1 px black outline, linear ticks every max/5."""
    return _make("gauge", value, title, min_val, max_val, height)


def create_horizontal_bar(value, title, min_val=0, max_val=100, height=400) -> Figure:
    """Horizontal bar (app.py:105-151): one bar, grid on x, hidden y labels and five
    translucent background rectangles below the bar."""
    return _make("bar", value, title, min_val, max_val, height)


def panel_spec(value, title, max_val, height, use_gauge=True) -> tuple:
    """A panel as a plain tuple (kind, value, title, min_val, max_val, height): what a
    dashboard refresh keeps per chart. ``figure_from_spec`` makes the Figure on demand
    (the Streamlit page); ``spec_json_parts`` serialises it without one."""
    if max_val == 0:
        raise ZeroDivisionError("division by zero")  # as get_color_for_value(value, 0)
    return ("gauge" if use_gauge else "bar", value, title, 0, max_val, height)


def figure_from_spec(spec) -> Figure:
    kind, value, title, min_val, max_val, height = spec
    return _make(kind, value, title, min_val, max_val, height)


def spec_json_parts(spec) -> tuple:
    """Figure JSON of a panel spec as 5 strings: cached template pieces + band colour +
    value (same bytes as ``figure_from_spec(spec).to_json()``)."""
    kind, value, title, min_val, max_val, height = spec
    head, mid, tail = _json_template(kind, title, min_val, max_val, height)
    return head, get_color_for_value(value, max_val), mid, _value_json(value), tail


def create_chart(value, title, max_val, height, use_gauge=True) -> Figure:
    """Style dispatch without any UI-framework state (the app layer supplies
    ``use_gauge`` from the session, app.py:242-245)."""
    if use_gauge:
        return create_gauge(value, title, max_val=max_val, height=height)
    return create_horizontal_bar(value, title, max_val=max_val, height=height)
