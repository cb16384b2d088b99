"""The Streamlit page: same layout, strings, widget keys and behaviour as the reference.

Reference: ``app.py:247-486`` (``main``), ``app.py:234-245`` (``create_visualization``).
Layout, in order: title + caption; "Display Settings" with the gauge toggle; "GPU
Selection" as a 4-column checkbox grid (keys ``gpu_checkbox_<id>``, first GPU selected
by default, stale selections dropped); debug sidebar; then a placeholder that is
redrawn every ``REFRESH_INTERVAL`` seconds with the average row, one row per
selected GPU, the statistics table and the "Last updated" footer.

Data sources (``ROCMDASH_DATA_SOURCE``):
  * ``prometheus`` (default): the reference's two PromQL queries against
    ``PROMETHEUS_METRICS_ENDPOINT`` (rocmdash.prom.query);
  * ``native``: one scrape per refresh of the local rank-per-GPU node service
    (``rocmdash.serve``, ``ROCMDASH_NODE_ENDPOINT``, default
    ``http://127.0.0.1:9400/metrics``): the RCCL-gathered node tensor - every series,
    window and node-window statistics, per-XCD detail - with no Prometheus between;
  * ``synthetic``: a synthetic 8-GPU node (demo / CPU).

The frame (figures, averages, tables) is built by ``rocmdash.viz.panels.build_frame``;
this module only maps it onto Streamlit calls.
"""

from __future__ import annotations

import os
import time
from datetime import datetime

from .. import config
from ..models.gpu_models import GPU_NAME_RESOLVE, GPU_POWER_LIMITS
from ..prom import query as _query
from ..viz.figures import (  # noqa: F401
    GAUGE_COLORS,
    create_gauge,
    create_horizontal_bar,
    figure_from_spec,
    get_color_for_value,
)
from ..viz.panels import NodeSnapshot, build_frame, natural_key, power_axis_max

PAGE_CONFIG = dict(
    page_title="GPU Metrics Dashboard",
    page_icon="📊",
    layout="wide",
    initial_sidebar_state="collapsed",
)


def _st():
    import streamlit as st

    return st


def get_power_limit(card_model):
    """``app.py:229-232`` (dead code in the reference, kept for API compatibility)."""
    resolved_model = GPU_NAME_RESOLVE.get(card_model, card_model)
    return GPU_POWER_LIMITS.get(resolved_model, GPU_POWER_LIMITS["default"])


def create_visualization(value, title, max_val, height, key, gpu_id=None, gpu_metrics_df=None):
    """Style dispatch (``app.py:234-245``): power panels use the GPU's power limit as
    the axis max; gauge or bar per ``st.session_state.use_gauge``. ``key`` is unused,
    as in the reference. ``gpu_metrics_df`` may be a DataFrame or a NodeSnapshot."""
    if title.endswith("Power Usage (W)") and gpu_id is not None and gpu_metrics_df is not None:
        if isinstance(gpu_metrics_df, NodeSnapshot):
            max_val = gpu_metrics_df.power_max(gpu_id)
        else:
            max_val = power_axis_max(gpu_metrics_df.loc[gpu_id, "card_model"])
    use_gauge = True
    try:
        use_gauge = bool(_st().session_state.use_gauge)
    except Exception:
        pass
    if use_gauge:
        return create_gauge(value, title, max_val=max_val, height=height)
    return create_horizontal_bar(value, title, max_val=max_val, height=height)


def fetch_gpu_metrics():
    """``app.py:153-227`` contract: ``(df, stats)`` or ``(None, None)`` + error banner."""
    return _query.fetch_gpu_metrics(on_error=lambda m: _st().error(m))


# ------------------------------------------------------------------ data sources
class _DataSource:
    _synthetic = None

    def __init__(self, kind: str | None = None):
        self.kind = (kind or os.environ.get("ROCMDASH_DATA_SOURCE", "prometheus")).lower()
        self.client = _query.PrometheusClient() if self.kind == "prometheus" else None

    def snapshot(self) -> NodeSnapshot:
        if self.kind == "prometheus":
            return _query.fetch_node_snapshot(self.client)
        if self.kind == "synthetic":
            from ..prom.exporter import SyntheticSource

            if _DataSource._synthetic is None:
                _DataSource._synthetic = SyntheticSource(int(os.environ.get("ROCMDASH_SYNTHETIC_GPUS", "8")))
            return _DataSource._synthetic.collect()[0]
        if self.kind == "native":
            return _query.fetch_service_snapshot()
        raise ValueError(f"unknown ROCMDASH_DATA_SOURCE {self.kind!r}")

    def fetch(self):
        """(snapshot | None); errors go to the banner like app.py:226."""
        try:
            return self.snapshot()
        except Exception as e:
            _st().error(f"Error fetching GPU metrics: {str(e)}")
            return None


def node_window_table(snap: NodeSnapshot) -> dict | None:
    """{series: {stat: value}} of the node-wide window statistics (None if absent)."""
    if snap.node_window is None:
        return None
    from ..models.schema import STAT_NAMES

    return {series: {k: round(float(snap.node_window[i, j]), 2) for j, k in enumerate(STAT_NAMES) if k != "last"}
            for i, series in enumerate(snap.window_series)}


def xcd_table(snap: NodeSnapshot, selected=None) -> dict | None:
    """{"GPU <id>": {"XCD <x> busy %": v, "XCD <x> MHz": v, ...}} of the selected GPUs'
    per-XCD detail (None if the data source has none)."""
    xcd = getattr(snap, "xcd", None)
    if xcd is None:
        return None
    sel = set(selected) if selected is not None else None
    table = {}
    for g, gid in enumerate(snap.gpu_ids):
        if sel is not None and gid not in sel:
            continue
        row = {}
        for x in range(xcd.shape[2]):
            if xcd[g, 0, x] != xcd[g, 0, x] and xcd[g, 1, x] != xcd[g, 1, x]:  # NaN: no such XCD
                continue
            row[f"XCD {x} busy %"] = float(xcd[g, 0, x])
            row[f"XCD {x} MHz"] = float(xcd[g, 1, x])
        if row:
            table[f"GPU {gid}"] = row
    return table or None


def _render_frame(st, frame, extended: bool, node_window: dict | None = None, xcd: dict | None = None) -> None:
    st.subheader("Average Metrics (Selected GPUs)")
    avg_cols = st.columns(4)
    for col, (key, spec) in zip(avg_cols, frame.avg_panels):
        with col:
            st.plotly_chart(figure_from_spec(spec).to_dict(), use_container_width=True, key=key)
    st.subheader("Individual GPU Metrics")
    for _, header, panels in frame.gpu_sections:
        st.markdown(header)
        ncols = 4
        for i in range(0, len(panels), ncols):
            cols = st.columns(ncols)
            for col, (key, spec) in zip(cols, panels[i : i + ncols]):
                with col:
                    st.plotly_chart(figure_from_spec(spec).to_dict(), use_container_width=True, key=key)
    st.subheader("GPU Metrics Statistics")
    import pandas as pd

    st.dataframe(pd.DataFrame(frame.stats_table), use_container_width=True)
    if extended and frame.window_table:
        st.subheader("Windowed Statistics (HIP window-stats kernel)")
        rows = {
            (gid, series): stats for gid, per in frame.window_table.items() for series, stats in per.items()
        }
        st.dataframe(pd.DataFrame.from_dict(rows, orient="index"), use_container_width=True)
    if extended and node_window is not None:
        st.subheader("Node-wide Windowed Statistics (all GPUs)")
        st.dataframe(pd.DataFrame(node_window), use_container_width=True)
    if extended and xcd is not None:
        st.subheader("Per-XCD Activity and Clocks")
        st.dataframe(pd.DataFrame.from_dict(xcd, orient="index"), use_container_width=True)
    st.text(frame.updated_text)


def main(max_refreshes: int | None = None, data_source: str | None = None) -> None:
    """The page. ``max_refreshes`` (or ``ROCMDASH_MAX_REFRESHES``) bounds the refresh
    loop for tests; the reference loops forever (``app.py:326``)."""
    st = _st()
    if max_refreshes is None and os.environ.get("ROCMDASH_MAX_REFRESHES"):
        max_refreshes = int(os.environ["ROCMDASH_MAX_REFRESHES"])
    extended = os.environ.get("ROCMDASH_EXTENDED", "0") not in ("0", "", "false")
    st.title("GPU Metrics Dashboard")
    st.markdown("Real-time monitoring of GPU metrics")

    if "selected_gpus" not in st.session_state:
        st.session_state.selected_gpus = []
    if "use_gauge" not in st.session_state:
        st.session_state.use_gauge = True

    st.header("Display Settings")
    use_gauge = st.toggle("Use Gauge Visualization", value=st.session_state.use_gauge)
    st.session_state.use_gauge = use_gauge

    source = _DataSource(data_source)
    snap = source.fetch()
    available_gpus = list(snap.gpu_ids) if snap is not None else []

    st.header("GPU Selection")
    num_columns = 4
    gpu_cols = st.columns(num_columns)
    if "last_selection" not in st.session_state:
        st.session_state.last_selection = None

    sorted_gpus = sorted(available_gpus, key=natural_key)
    st.session_state.selected_gpus = [g for g in st.session_state.selected_gpus if g in sorted_gpus]
    if not st.session_state.selected_gpus and sorted_gpus:
        st.session_state.selected_gpus = [sorted_gpus[0]]

    for i, gpu_id in enumerate(sorted_gpus):
        with gpu_cols[i % num_columns]:
            is_currently_selected = gpu_id in st.session_state.selected_gpus
            is_selected = st.checkbox(f"GPU {gpu_id}", value=is_currently_selected, key=f"gpu_checkbox_{gpu_id}")
            if is_selected != is_currently_selected:
                if is_selected:
                    st.session_state.selected_gpus.append(gpu_id)
                else:
                    st.session_state.selected_gpus.remove(gpu_id)
                st.session_state.last_selection = gpu_id

    st.session_state.selected_gpus.sort(key=natural_key)

    st.sidebar.write("Debug Info:")
    st.sidebar.write("Current selections:", st.session_state.selected_gpus)
    st.sidebar.write("Last selection:", st.session_state.last_selection)

    placeholder = st.empty()
    n = 0
    while max_refreshes is None or n < max_refreshes:
        now = datetime.now()
        with placeholder.container():
            snap = source.fetch()
            if snap is not None:
                frame = build_frame(
                    snap, st.session_state.selected_gpus, use_gauge=st.session_state.use_gauge, extended=extended, now=now
                )
                _render_frame(st, frame, extended, node_window_table(snap) if extended else None,
                              xcd_table(snap, st.session_state.selected_gpus) if extended else None)
        n += 1
        if max_refreshes is not None and n >= max_refreshes:
            break
        time.sleep(config.REFRESH_INTERVAL)
