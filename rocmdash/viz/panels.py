"""One dashboard refresh ("frame"): node snapshot -> averages, per-GPU panels, tables.

Reference: the body of the refresh loop, ``app.py:326-486``:
  * selected-GPU averages, power mean over non-zero readings only (``app.py:335-345``);
  * 4 average panels (``app.py:348-409``), then per selected GPU a
    ``### GPU <id> (<model>)`` header and 4 panels (``app.py:412-476``);
  * the mean/max/min statistics table over ALL GPUs, rounded to 2 places
    (``app.py:216-221, 479-481``) and the "Last updated" footer (``app.py:484``).

The frame is UI-framework independent: the Streamlit page (``rocmdash.ui.page``)
renders it element by element, and ``Frame.to_json`` produces the whole refresh
payload in one go (what the benchmark times, BASELINE.md "full refresh latency").

Differences from the reference, all within SURVEY.md §7.1's "reasonable fixes":
  * metric columns are float64 (the reference's pivot leaves them object dtype);
  * a selected GPU that vanished is skipped instead of raising ``KeyError``
    (``app.py:335``);
  * the power-axis max prefers the power cap amd-smi reports for that GPU and falls
    back to the reference's model table (``app.py:236-240``);
  * optional extended rows: MFMA utilisation, HBM read/write bandwidth and the
    windowed p50/p90/p99 table computed by the HIP window-stats kernel.
"""

from __future__ import annotations

import json
import math
import re
import time
from dataclasses import dataclass, field
from datetime import datetime

import numpy as np

from ..models.gpu_models import GPU_NAME_RESOLVE, GPU_POWER_LIMITS, resolve_model
from ..models.health import SourceHealth
from ..models.schema import COMPAT_METRICS, STAT_NAMES
from .figures import Figure, figure_from_spec, panel_spec, spec_json_parts

VRAM_RATIO = "vram_usage_ratio"
POWER = "amd_gpu_average_package_power"
UTIL = "amd_gpu_gfx_activity"
TEMP = "amd_gpu_edge_temperature"
USED = "amd_gpu_used_vram"
TOTAL = "amd_gpu_total_vram"

HEIGHT_AVERAGE = 300  # app.py:323
HEIGHT_SPECIFIC = 200  # app.py:324

_NAT = re.compile(r"(\d+)")


def natural_key(s):
    """'10' sorts after '2' (the reference sorts lexicographically, app.py:277)."""
    return [int(t) if t.isdigit() else t for t in _NAT.split(str(s))]


def power_axis_max(card_model, power_limit_w=None):
    """Power gauge max: amd-smi's cap for that GPU when known, else the reference's
    part-number -> model -> limit table with its 300 W default (app.py:236-240)."""
    if power_limit_w is not None and power_limit_w == power_limit_w and power_limit_w > 0:
        return float(power_limit_w)
    resolved = GPU_NAME_RESOLVE.get(card_model, card_model)
    if resolved not in GPU_POWER_LIMITS:
        hinted = resolve_model(card_model)
        if hinted is not None:
            resolved = hinted
    return GPU_POWER_LIMITS.get(resolved, GPU_POWER_LIMITS["default"])


@dataclass
class NodeSnapshot:
    """Latest value of every metric of every GPU of the node (+ optional window stats).

    ``values[g, c]`` is the newest sample of ``columns[c]`` on GPU ``gpu_ids[g]``;
    ``window[g, s, k]`` is statistic ``STAT_NAMES[k]`` of series ``window_series[s]``
    over the last W samples (the HIP kernel's output, all-gathered over the node);
    ``node_window[s, k]`` the same over the union of all GPUs' windows.
    """

    gpu_ids: list
    card_models: list
    columns: tuple
    values: np.ndarray
    power_limits: list = field(default_factory=list)
    product_names: list = field(default_factory=list)
    window: np.ndarray | None = None
    window_series: tuple = ()
    timestamp: float = field(default_factory=time.time)
    # [S, 8] statistics of each window series over every GPU's window at once
    # (rocmdash.parallel.node_window), when computed
    node_window: np.ndarray | None = None
    # [N, 2, XCDS] per-XCD busy (%) and gfx clock (MHz) of each GPU's latest SMU
    # sample, when the data source has it
    xcd: np.ndarray | None = None
    # every GPU's per-source sampler health (rocmdash.models.health), when known
    source_health: SourceHealth | None = None
    # Unix time of the node refresh that produced these values (the node service's
    # rocmdash_node_refresh_timestamp_seconds), when the data source exports it: a
    # sample's own time is refresh_time - its source's age_s
    refresh_time: float | None = None

    def __post_init__(self):
        self.values = np.asarray(self.values, dtype=np.float64)
        if self.values.size == 0:
            self.values = self.values.reshape(len(self.gpu_ids), len(self.columns))
        if self.values.shape != (len(self.gpu_ids), len(self.columns)):
            raise ValueError(f"values shape {self.values.shape} != ({len(self.gpu_ids)}, {len(self.columns)})")
        self.gpu_ids = [str(g) for g in self.gpu_ids]
        if not self.power_limits:
            self.power_limits = [None] * len(self.gpu_ids)
        if not self.product_names:
            self.product_names = [None] * len(self.gpu_ids)
        self._col = {c: i for i, c in enumerate(self.columns)}
        self._row = {g: i for i, g in enumerate(self.gpu_ids)}
        if VRAM_RATIO not in self._col and USED in self._col and TOTAL in self._col:
            with np.errstate(divide="ignore", invalid="ignore"):
                ratio = self.values[:, self._col[USED]] / self.values[:, self._col[TOTAL]] * 100.0
            self.values = np.concatenate([self.values, ratio[:, None]], axis=1)
            self.columns = tuple(self.columns) + (VRAM_RATIO,)
            self._col[VRAM_RATIO] = len(self.columns) - 1

    # -------------------------------------------------------------- accessors
    def has(self, col) -> bool:
        return col in self._col

    def row(self, gpu_id) -> int:
        return self._row[str(gpu_id)]

    def value(self, gpu_id, col, default=0.0):
        c = self._col.get(col)
        if c is None:
            return default
        return float(self.values[self._row[str(gpu_id)], c])

    def sorted_gpu_ids(self, natural=True):
        return sorted(self.gpu_ids, key=natural_key if natural else None)

    def card_model(self, gpu_id):
        return self.card_models[self._row[str(gpu_id)]]

    def model_name(self, gpu_id):
        r = self._row[str(gpu_id)]
        return resolve_model(self.card_models[r], self.product_names[r])

    def power_max(self, gpu_id):
        r = self._row[str(gpu_id)]
        return power_axis_max(self.card_models[r], self.power_limits[r])

    # -------------------------------------------------------------- statistics
    def stats(self) -> dict:
        """mean/max/min over ALL GPUs of every numeric column (app.py:216-221); NaNs
        are skipped like pandas does."""
        mean, mx, mn = _nan_mean_max_min(self.values)
        return {
            "mean": dict(zip(self.columns, mean.tolist())),
            "max": dict(zip(self.columns, mx.tolist())),
            "min": dict(zip(self.columns, mn.tolist())),
        }

    # -------------------------------------------------------------- pandas views
    def to_dataframe(self):
        """The reference's ``(df_pivot, stats)`` contract (app.py:204-223): index =
        string gpu_id named 'gpu_id', metric columns (sorted, as pivot sorts them) plus
        ``card_model`` and ``vram_usage_ratio`` last; stats = dict of Series."""
        import pandas as pd

        base = sorted(c for c in self.columns if c != VRAM_RATIO)
        cols = {c: self.values[:, self._col[c]] for c in base}
        df = pd.DataFrame(cols, index=pd.Index(self.gpu_ids, name="gpu_id"))
        df.insert(sorted(base + ["card_model"]).index("card_model"), "card_model", list(self.card_models))
        df.columns.name = "metric_name"
        if VRAM_RATIO in self._col:
            df[VRAM_RATIO] = self.values[:, self._col[VRAM_RATIO]]
        numeric = [c for c in df.columns if c != "card_model"]
        stats = {"mean": df[numeric].mean(), "max": df[numeric].max(), "min": df[numeric].min()}
        return df, stats

    @classmethod
    def from_dataframe(cls, df, power_limits=None, window=None, window_series=()):
        cols = tuple(c for c in df.columns if c not in ("card_model", VRAM_RATIO))
        values = df[list(cols)].to_numpy(dtype=np.float64) if cols else np.zeros((len(df), 0))
        cms = df["card_model"].tolist() if "card_model" in df.columns else [None] * len(df)
        return cls(
            gpu_ids=[str(i) for i in df.index],
            card_models=cms,
            columns=cols,
            values=values,
            power_limits=list(power_limits or []),
            window=window,
            window_series=tuple(window_series),
        )


def _nan_mean_max_min(v: np.ndarray):
    """Column-wise NaN-skipping mean / max / min without numpy's warning machinery
    (an all-NaN column gives NaN, as pandas does)."""
    if not len(v):
        nan = np.full(v.shape[1], np.nan)
        return nan, nan, nan
    valid = ~np.isnan(v)
    cnt = valid.sum(axis=0)
    with np.errstate(invalid="ignore", divide="ignore"):
        mean = np.where(valid, v, 0.0).sum(axis=0) / cnt
    mx = np.fmax.reduce(v, axis=0)
    mn = np.fmin.reduce(v, axis=0)
    return mean, mx, mn


def selected_averages(snap: NodeSnapshot, selected) -> dict:
    """Means over the selected GPUs; the power mean ignores zero readings when any
    reading is non-zero (app.py:338-345)."""
    rows = [snap._row[str(g)] for g in selected if str(g) in snap._row]
    if not rows:
        return {c: float("nan") for c in snap.columns}
    sub = snap.values[rows]
    means = _nan_mean_max_min(sub)[0]
    out = dict(zip(snap.columns, means.tolist()))
    if POWER in snap._col:
        p = sub[:, snap._col[POWER]]
        nz = p[p > 0]
        if nz.size:
            out[POWER] = float(nz.mean())
    return out


def _json_numbers(a) -> str:
    """JSON of a (nested) float array rounded to 2 places; NaN/inf -> null."""
    r = np.round(np.asarray(a, dtype=np.float64), 2)
    r[~np.isfinite(r)] = np.nan
    return json.dumps(r.tolist()).replace("NaN", "null")


WINDOW_STATS = ("p50", "p90", "p99", "min", "max", "mean")


@dataclass
class Frame:
    """Everything one refresh shows, in display order."""

    timestamp_key: str
    updated_text: str
    averages: dict
    avg_panels: list  # [(plot_key, panel spec)] x4 (viz.figures.panel_spec)
    gpu_sections: list  # [(gpu_id, header_markdown, [(plot_key, panel spec)] x4 or x7)]
    stats_columns: tuple  # numeric columns of the statistics table
    stats_values: np.ndarray  # [3, C]: mean / max / min over all GPUs
    window_gpus: tuple = ()
    window_series: tuple = ()
    window_values: np.ndarray | None = None  # [G, S, len(WINDOW_STATS)]

    def panels(self):
        """(plot_key, panel spec) of every chart in display order."""
        yield from self.avg_panels
        for _, _, panels in self.gpu_sections:
            yield from panels

    def figures(self):
        """(plot_key, Figure) of every chart in display order (built on demand)."""
        for key, spec in self.panels():
            yield key, figure_from_spec(spec)

    @property
    def num_figures(self) -> int:
        return len(self.avg_panels) + sum(len(p) for _, _, p in self.gpu_sections)

    @property
    def stats_table(self) -> dict:
        """{"mean"|"max"|"min": {column: value rounded to 2 (None for NaN)}}."""
        r = np.round(self.stats_values, 2)
        return {
            k: {c: (None if not math.isfinite(x) else x) for c, x in zip(self.stats_columns, r[i].tolist())}
            for i, k in enumerate(("mean", "max", "min"))
        }

    @property
    def window_table(self) -> dict | None:
        """{gpu_id: {series: {stat: value}}} of the window statistics (UI table)."""
        if self.window_values is None:
            return None
        r = np.round(self.window_values, 2).tolist()
        return {
            g: {
                s: {k: (None if not math.isfinite(x) else x) for k, x in zip(WINDOW_STATS, r[gi][si])}
                for si, s in enumerate(self.window_series)
            }
            for gi, g in enumerate(self.window_gpus)
        }

    def to_json(self) -> str:
        """The whole refresh payload: every figure's Plotly JSON + tables + footer.
        Tables are columnar: {"columns": [...], "rows": [...], "values": [[...]]}."""
        parts = ['{"updated":', json.dumps(self.updated_text), ',"figures":{']
        first = True
        for key, spec in self.panels():
            if not first:
                parts.append(",")
            first = False
            parts.append('"' + key + '":' if key.isascii() and '"' not in key and "\\" not in key else json.dumps(key) + ":")
            parts.extend(spec_json_parts(spec))
        parts.append('},"headers":')
        parts.append(json.dumps([h for _, h, _ in self.gpu_sections]))
        parts.append(',"stats":{"rows":["mean","max","min"],"columns":')
        parts.append(json.dumps(list(self.stats_columns)))
        parts.append(',"values":')
        parts.append(_json_numbers(self.stats_values))
        parts.append("}")
        if self.window_values is not None:
            parts.append(',"window":{"gpus":')
            parts.append(json.dumps(list(self.window_gpus)))
            parts.append(',"series":')
            parts.append(json.dumps(list(self.window_series)))
            parts.append(',"stats":')
            parts.append(json.dumps(list(WINDOW_STATS)))
            parts.append(',"values":')
            parts.append(_json_numbers(self.window_values))
            parts.append("}")
        parts.append("}")
        return "".join(parts)


_WINDOW_IDX = [STAT_NAMES.index(k) for k in WINDOW_STATS]


EXTENDED_PANELS = (
    ("amd_gpu_cu_active", "CU Active (%)", "cu_active", 100.0),
    ("amd_gpu_mfma_utilization", "MFMA Utilization (%)", "mfma_util", 100.0),
    # memory-side traffic (HBM + Infinity Cache hits); axis = the HBM peak
    ("amd_gpu_hbm_read_bandwidth", "HBM/MALL Read (GB/s)", "hbm_read", 8000.0),
    ("amd_gpu_hbm_write_bandwidth", "HBM/MALL Write (GB/s)", "hbm_write", 8000.0),
    ("amd_gpu_xgmi_read_bandwidth", "xGMI Receive (GB/s)", "xgmi_read", 600.0),
    ("amd_gpu_xgmi_write_bandwidth", "xGMI Send (GB/s)", "xgmi_write", 600.0),
)


_PRESENT_CACHE: dict = {}


def _present(snap: NodeSnapshot, selected, natural_sort: bool) -> list:
    """Selected GPUs that the snapshot has, in display order (memoised: the same
    selection over the same GPUs is asked for every refresh)."""
    key = (tuple(selected), tuple(snap.gpu_ids), natural_sort)
    hit = _PRESENT_CACHE.get(key)
    if hit is not None:
        return list(hit)
    present = [str(g) for g in selected if str(g) in snap._row]
    present.sort(key=natural_key if natural_sort else None)
    if len(_PRESENT_CACHE) > 256:
        _PRESENT_CACHE.clear()
    _PRESENT_CACHE[key] = tuple(present)
    return present


# value sources of a panel: a GPU's own value, the selected-GPU average, or the
# reference's literal 0 for a metric the node does not report
SRC_ROW, SRC_AVG, SRC_ZERO = 0, 1, 2


def _layout(snap: NodeSnapshot, present: list, extended: bool) -> tuple:
    """The refresh's panel layout, shared by the Python and the native renderer:
    ``(avg_panels, sections)`` with panels ``(key_prefix, title, max_val, height, src,
    row, col)`` and sections ``(gpu_id, header, panels)`` (app.py:348-476)."""
    first = present[0] if present else None
    power_max = snap.power_max(first) if first is not None else 300

    def avg(name):
        c = snap._col.get(name)
        return (SRC_ZERO, -1, 0) if c is None else (SRC_AVG, -1, c)

    avg_panels = [
        ("plot_avg_gpu_util_", "Avg GPU Utilization (%)", 100, HEIGHT_AVERAGE) + avg(UTIL),
        ("plot_avg_vram_usage_", "Avg VRAM Usage (%)", 100, HEIGHT_AVERAGE) + avg(VRAM_RATIO),
        ("plot_avg_temp_", "Avg Temperature (°C)", 100, HEIGHT_AVERAGE) + avg(TEMP),
        ("plot_avg_power_", "Avg Power Usage (W)", power_max, HEIGHT_AVERAGE) + avg(POWER),
    ]
    sections = []
    for gid in present:
        r = snap._row[gid]

        def v(name):
            c = snap._col.get(name)
            return (SRC_ZERO, r, 0) if c is None else (SRC_ROW, r, c)

        panels = [
            (f"plot_gpu_util_{gid}_", "GPU Utilization (%)", 100, HEIGHT_SPECIFIC) + v(UTIL),
            (f"plot_vram_usage_{gid}_", "VRAM Usage (%)", 100, HEIGHT_SPECIFIC) + v(VRAM_RATIO),
            (f"plot_temp_{gid}_", "Temperature (°C)", 100, HEIGHT_SPECIFIC) + v(TEMP),
            (f"plot_power_{gid}_", "Power Usage (W)", snap.power_max(gid), HEIGHT_SPECIFIC) + v(POWER),
        ]
        if extended:
            for col, title, key, mx in EXTENDED_PANELS:
                if snap.has(col):
                    panels.append((f"plot_{key}_{gid}_", title, mx, HEIGHT_SPECIFIC) + v(col))
        sections.append((gid, f"### GPU {gid} ({snap.model_name(gid)})", panels))
    return avg_panels, sections


def build_frame(
    snap: NodeSnapshot,
    selected,
    use_gauge: bool = True,
    extended: bool = False,
    now: datetime | None = None,
    natural_sort: bool = True,
    window_table: bool | None = None,
) -> Frame:
    """Build one refresh of the dashboard for the selected GPUs (app.py:326-484).

    ``window_table`` (default: ``extended``) adds the windowed-statistics table the
    extended page shows; the reference panel set has none."""
    with_window = extended if window_table is None else window_table
    with_window = with_window and snap.window is not None and len(snap.window_series) > 0
    now = now or datetime.now()
    ts = now.strftime("%Y%m%d%H%M%S%f")
    present = _present(snap, selected, natural_sort)
    avg = selected_averages(snap, present)
    avg_by_col = [avg[c] for c in snap.columns]
    avg_layout, sec_layout = _layout(snap, present, extended)

    def spec(panel):
        prefix, title, max_val, height, src, row, col = panel
        if src == SRC_ROW:
            value = float(snap.values[row, col])
        elif src == SRC_AVG:
            value = avg_by_col[col]
            value = 0 if value is None else value
        else:
            value = 0
        return prefix + ts, panel_spec(value, title, max_val, height, use_gauge)

    return Frame(
        timestamp_key=ts,
        updated_text=f"Last updated: {now.strftime('%Y-%m-%d %H:%M:%S')}",
        averages=avg,
        avg_panels=[spec(p) for p in avg_layout],
        gpu_sections=[(gid, header, [spec(p) for p in panels]) for gid, header, panels in sec_layout],
        stats_columns=tuple(snap.columns),
        stats_values=np.stack(_nan_mean_max_min(snap.values)),
        window_gpus=tuple(snap.gpu_ids) if with_window else (),
        window_series=tuple(snap.window_series) if with_window else (),
        window_values=snap.window[:, :, _WINDOW_IDX] if with_window else None,
    )


# ------------------------------------------------------------------ native renderer
_PLAN_CACHE: dict = {}
_native_render = None  # None = not probed, False = unavailable, else the module


def _native():
    global _native_render
    if _native_render is None:
        try:
            from ..runtime.native import load

            mod = load()
            _native_render = mod if hasattr(mod, "render_frame") else False
        except Exception:
            _native_render = False
    return _native_render


def _safe_key(k: str) -> bool:
    return k.isascii() and '"' not in k and "\\" not in k


def _compile_plan(nat, snap: NodeSnapshot, present: list, use_gauge: bool, extended: bool, with_window: bool):
    from .figures import _json_template

    kind = "gauge" if use_gauge else "bar"
    avg_layout, sec_layout = _layout(snap, present, extended)
    panels = []
    for prefix, title, max_val, height, src, row, col in avg_layout + [p for _, _, ps in sec_layout for p in ps]:
        if not _safe_key(prefix):
            return None
        if max_val == 0:
            raise ZeroDivisionError("division by zero")
        head, mid, tail = _json_template(kind, title, 0, max_val, height)
        panels.append((prefix, head, mid, tail, float(max_val), src, row, col))
    power_col = snap._col.get(POWER, -1)
    return nat.FramePlan(
        panels=panels,
        sel_rows=[snap._row[g] for g in present],
        power_col=power_col,
        headers_json=json.dumps([h for _, h, _ in sec_layout]),
        stats_columns_json=json.dumps(list(snap.columns)),
        num_columns=len(snap.columns),
        window=with_window,
        window_gpus_json=json.dumps(list(snap.gpu_ids)),
        window_series_json=json.dumps(list(snap.window_series)),
        window_stats_json=json.dumps(list(WINDOW_STATS)),
        window_stat_idx=list(_WINDOW_IDX),
        window_series=len(snap.window_series),
    )


def render_frame_json(
    snap: NodeSnapshot,
    selected,
    use_gauge: bool = True,
    extended: bool = False,
    now: datetime | None = None,
    natural_sort: bool = True,
    window_table: bool | None = None,
    native: bool | None = None,
) -> str:
    """``build_frame(...).to_json()`` - through the native renderer when available
    (byte-identical output, GIL released while rendering; tests/test_frame_render.py).
    The layout is compiled once per (GPU set, selection, style) and cached."""
    nat = _native() if native is not False else False
    if not nat:
        if native:
            raise RuntimeError("native frame renderer unavailable")
        return build_frame(snap, selected, use_gauge, extended, now, natural_sort, window_table).to_json()
    with_window = extended if window_table is None else window_table
    with_window = bool(with_window and snap.window is not None and len(snap.window_series) > 0)
    present = _present(snap, selected, natural_sort)
    key = (
        tuple(snap.gpu_ids), tuple(snap.columns), tuple(snap.card_models), tuple(snap.power_limits),
        tuple(snap.product_names), tuple(present), bool(use_gauge), bool(extended), with_window,
        tuple(snap.window_series),
    )
    plan = _PLAN_CACHE.get(key)
    if plan is None:
        plan = _compile_plan(nat, snap, present, use_gauge, extended, with_window)
        if plan is None:  # a key the native path does not escape: Python path
            return build_frame(snap, selected, use_gauge, extended, now, natural_sort, window_table).to_json()
        if len(_PLAN_CACHE) > 64:
            _PLAN_CACHE.clear()
        _PLAN_CACHE[key] = plan
    ts, updated = _time_strings(now)
    window = snap.window if with_window else None
    return nat.render_frame(plan, snap.values, window, ts, updated)


_TS_CACHE = [None, "", ""]  # second, "%Y%m%d%H%M%S", json "Last updated: ..."


def _time_strings(now: datetime | None = None) -> tuple:
    """(plot-key timestamp "%Y%m%d%H%M%S%f", JSON footer) of ``now`` (default: the
    local time now); the per-second parts are formatted once per second."""
    if now is None:
        t = time.time()
        sec = int(t)
        us = int((t - sec) * 1e6)
        if _TS_CACHE[0] != sec:
            d = datetime.fromtimestamp(sec)
            _TS_CACHE[:] = [sec, d.strftime("%Y%m%d%H%M%S"), json.dumps(f"Last updated: {d.strftime('%Y-%m-%d %H:%M:%S')}")]
        return f"{_TS_CACHE[1]}{us:06d}", _TS_CACHE[2]
    return now.strftime("%Y%m%d%H%M%S%f"), json.dumps(f"Last updated: {now.strftime('%Y-%m-%d %H:%M:%S')}")


class CompiledFrame:
    """The native renderer bound to one node layout, for refresh loops whose GPUs,
    series, models, selection and style do not change (rocmdash/runtime/pipeline.py):
    the plan is compiled once and each refresh goes straight from the gathered
    ``[N, S, 8]`` stats to the payload - no NodeSnapshot, no selection sort, no plan
    lookup. Payloads are byte-identical to ``render_frame_json`` of the equivalent
    snapshot (tests/test_frame_render.py)."""

    def __init__(self, snap: NodeSnapshot, selected, use_gauge: bool = True, extended: bool = False,
                 natural_sort: bool = True, window_table: bool | None = None):
        nat = _native()
        if not nat:
            raise RuntimeError("native frame renderer unavailable")
        with_window = extended if window_table is None else window_table
        self.with_window = bool(with_window and snap.window is not None and len(snap.window_series) > 0)
        present = _present(snap, selected, natural_sort)
        self.plan = _compile_plan(nat, snap, present, use_gauge, extended, self.with_window)
        if self.plan is None:
            raise RuntimeError("layout not renderable natively")
        self._nat = nat
        self.columns = tuple(snap.columns)
        self.num_gpus = len(snap.gpu_ids)
        self._values = np.empty((self.num_gpus, len(self.columns)), dtype=np.float64)
        col = {c: i for i, c in enumerate(self.columns)}
        self._ratio = (col[VRAM_RATIO], col[USED], col[TOTAL]) if all(k in col for k in (VRAM_RATIO, USED, TOTAL)) else None

    def render(self, last: np.ndarray, window: np.ndarray | None = None, now: datetime | None = None,
               as_bytes: bool = False):
        """``last``: [G, S] newest values (S = the snapshot's series without derived
        columns); ``window``: [G, S, 8] stats for the window table."""
        v = self._values
        S = last.shape[1]
        v[:, :S] = last
        if self._ratio is not None:
            r, u, t = self._ratio
            tot = v[:, t]
            if (tot != 0).all():
                np.multiply(v[:, u] / tot, 100.0, out=v[:, r])
            else:
                with np.errstate(divide="ignore", invalid="ignore"):
                    v[:, r] = v[:, u] / tot * 100.0
        ts, updated = _time_strings(now)
        return self._nat.render_frame(self.plan, v, window if self.with_window else None, ts, updated, as_bytes)


__all__ = [
    "SourceHealth",
    "COMPAT_METRICS",
    "Frame",
    "NodeSnapshot",
    "build_frame",
    "render_frame_json",
    "CompiledFrame",
    "natural_key",
    "power_axis_max",
    "selected_averages",
    "Figure",
]
