"""Series -> ``NodeSnapshot``: the inverse of ``exposition.render_snapshot``.

One builder for every place the dashboard reads labelled samples back:

  * Prometheus mode with ``ROCMDASH_EXTENDED=1`` (``query.fetch_node_snapshot``): the
    reference's compat query (``app.py:167-172``, kept byte-identical) plus ONE more
    instant query for the extended series, window statistics, node-window statistics,
    per-XCD detail and per-source health the node service exports;
  * ``native`` mode of the page (``ui/page.py``): a direct scrape of the local
    rank-per-GPU node service's ``/metrics`` (``rocmdash.serve``), so the page shows
    exactly the RCCL-gathered node tensor, without a Prometheus in between.

Input items are ``(labels, value)`` with the metric name in ``labels["__name__"]`` -
the shape of a Prometheus instant-vector result and of a parsed exposition sample.
"""

from __future__ import annotations

import math

import numpy as np

from ..models.health import SourceHealth
from ..models.schema import (
    COMPAT_METRICS,
    HEALTH_INDEX,
    HEALTH_SOURCES,
    HEALTH_SPLIT,
    METRIC_SPECS,
    NUM_STATS,
    STAT_INDEX,
    XCDS,
)
from ..viz.panels import NodeSnapshot, natural_key

# every amd_gpu_* value series the exporter publishes, compat ones first
VALUE_SERIES = COMPAT_METRICS + tuple(m for m in METRIC_SPECS if m not in COMPAT_METRICS)
EXTENDED_SERIES = tuple(m for m in METRIC_SPECS if m not in COMPAT_METRICS)
WINDOW_NAMES = ("rocmdash_window", "rocmdash_window_samples", "rocmdash_node_window")
XCD_NAMES = ("amd_gpu_xcd_activity", "amd_gpu_xcd_gfx_clock")
HEALTH_NAMES = ("rocmdash_sampler_samples_total", "rocmdash_sampler_failures_total", "rocmdash_sampler_overruns_total",
                "rocmdash_sample_age_seconds", "rocmdash_sampler_rate_hz")
REFRESH_TS = "rocmdash_node_refresh_timestamp_seconds"


def extended_query(node_ip: str) -> str:
    """The one extra instant query of the extended view (everything the node service
    exports per GPU beyond the reference's five series), on the same instance filter
    as ``app.py:171``."""
    names = EXTENDED_SERIES + ("amd_gpu_power_cap", "amd_gpu_info") + WINDOW_NAMES + XCD_NAMES + HEALTH_NAMES + (REFRESH_TS,)
    return "{__name__=~\"" + "|".join(names) + "\", instance=~\"" + node_ip + ":.+\"}"


def _put(table: dict, gid: str, key, value: float) -> None:
    row = table.setdefault(gid, {})
    if key in row:  # same contract as the reference's pivot (app.py:204-207)
        raise ValueError("Index contains duplicate entries, cannot reshape")
    row[key] = value


def snapshot_from_series(items, require_vram: bool = True) -> NodeSnapshot:
    """Build a snapshot from ``(labels, value)`` items (see module doc). Raises like
    the reference's pivot on duplicate (gpu, series) and on missing VRAM columns."""
    values: dict = {}
    models: dict = {}
    power: dict = {}
    product: dict = {}
    window: dict = {}  # gid -> {(series, stat): v}
    node_window: dict = {}
    xcd: dict = {}
    health: dict = {}  # gid -> {(source, field): v}
    backends: dict = {}  # gid -> {source: backend}
    names = set()
    refresh_time = None
    for labels, v in items:
        name = labels.get("__name__", "")
        v = float(v)
        gid = labels.get("gpu_id")
        if name == REFRESH_TS:
            refresh_time = v if refresh_time is None else max(refresh_time, v)
            continue
        if name == "rocmdash_node_window":
            key = (labels.get("metric", ""), labels.get("stat", ""))
            node_window[key] = v  # one series set per node; duplicates across ports: last wins
            continue
        if gid is None:
            continue
        if gid not in models and "card_model" in labels:
            models[gid] = labels["card_model"]
        if name in METRIC_SPECS:
            _put(values, gid, name, v)
            names.add(name)
        elif name == "amd_gpu_power_cap":
            power[gid] = v
        elif name == "amd_gpu_info":
            product[gid] = labels.get("product_name", "")
        elif name == "rocmdash_window":
            _put(window, gid, (labels.get("metric", ""), labels.get("stat", "")), v)
        elif name == "rocmdash_window_samples":
            _put(window, gid, (labels.get("metric", ""), "count"), v)
        elif name in XCD_NAMES:
            try:
                x = int(labels.get("xcd", ""))
            except ValueError:
                continue
            if 0 <= x < XCDS:
                _put(xcd, gid, (XCD_NAMES.index(name), x), v)
        elif name in HEALTH_NAMES:
            src = labels.get("source", "")
            if src in HEALTH_SOURCES:
                _put(health, gid, (src, name), v)
                backends.setdefault(gid, {})[src] = labels.get("backend", "")
    if require_vram:
        for req in ("amd_gpu_used_vram", "amd_gpu_total_vram"):
            if req not in names:
                raise KeyError(req)
    gpu_ids = sorted(values, key=natural_key)
    columns = tuple(c for c in VALUE_SERIES if c in names)
    vals = np.array([[values[g].get(c, math.nan) for c in columns] for g in gpu_ids], dtype=np.float64)
    snap = NodeSnapshot(
        gpu_ids=gpu_ids,
        card_models=[models.get(g, "") for g in gpu_ids],
        columns=columns,
        values=vals.reshape(len(gpu_ids), len(columns)),
        power_limits=[power.get(g) for g in gpu_ids],
        product_names=[product.get(g, "") for g in gpu_ids],
        refresh_time=refresh_time,
    )
    wnames = {s for per in window.values() for s, _ in per}
    wseries = tuple(c for c in VALUE_SERIES if c in wnames)
    if wseries:
        w = np.full((len(gpu_ids), len(wseries), NUM_STATS), np.nan, dtype=np.float32)
        for gi, g in enumerate(gpu_ids):
            per = window.get(g, {})
            for si, s in enumerate(wseries):
                for stat, k in STAT_INDEX.items():
                    if (s, stat) in per:
                        w[gi, si, k] = per[(s, stat)]
                w[gi, si, STAT_INDEX["last"]] = values[g].get(s, math.nan)
        snap.window = w
        snap.window_series = wseries
    if node_window:
        series = snap.window_series or tuple(dict.fromkeys(s for s, _ in node_window))
        nw = np.full((len(series), NUM_STATS), np.nan)
        for si, s in enumerate(series):
            for stat, k in STAT_INDEX.items():
                if (s, stat) in node_window:
                    nw[si, k] = node_window[(s, stat)]
        snap.node_window = nw
        if not snap.window_series:
            snap.window_series = series
    if xcd:
        arr = np.full((len(gpu_ids), 2, XCDS), np.nan, dtype=np.float32)
        for gi, g in enumerate(gpu_ids):
            for (k, x), v in xcd.get(g, {}).items():
                arr[gi, k, x] = v
        snap.xcd = arr
    if health:
        H = HEALTH_INDEX
        rows = np.full((len(gpu_ids), len(HEALTH_SOURCES), NUM_STATS), np.nan)
        for gi, g in enumerate(gpu_ids):
            per = health.get(g, {})
            for i, src in enumerate(HEALTH_SOURCES):
                rows[gi, i, H["present"]] = 0.0
                if (src, "rocmdash_sampler_samples_total") not in per:
                    continue
                for fam, hi, lo in (("rocmdash_sampler_samples_total", "samples_hi", "samples_lo"),
                                    ("rocmdash_sampler_failures_total", "failures_hi", "failures_lo")):
                    rows[gi, i, H[hi]], rows[gi, i, H[lo]] = divmod(per.get((src, fam), 0.0), HEALTH_SPLIT)
                rows[gi, i, H["overruns"]] = per.get((src, "rocmdash_sampler_overruns_total"), 0.0)
                rows[gi, i, H["age_s"]] = per.get((src, "rocmdash_sample_age_seconds"), math.nan)
                rows[gi, i, H["hz"]] = per.get((src, "rocmdash_sampler_rate_hz"), math.nan)
                rows[gi, i, H["present"]] = 1.0
        snap.source_health = SourceHealth(
            rows, [tuple(backends.get(g, {}).get(s, "") for s in HEALTH_SOURCES) for g in gpu_ids])
    return snap


def merge_extended(base: NodeSnapshot, ext: NodeSnapshot) -> NodeSnapshot:
    """The compat snapshot (the reference's query, its GPU set and error semantics)
    widened with the extended query's columns, window, node window, XCD and health."""
    if not ext.gpu_ids:
        return base
    cols = list(base.columns)
    extra = [c for c in ext.columns if c not in base.columns]
    vals = np.full((len(base.gpu_ids), len(cols) + len(extra)), np.nan)
    vals[:, : len(cols)] = base.values
    rows = [ext.gpu_ids.index(g) if g in ext.gpu_ids else -1 for g in base.gpu_ids]
    for j, c in enumerate(extra):
        ci = ext.columns.index(c)
        for gi, r in enumerate(rows):
            if r >= 0:
                vals[gi, len(cols) + j] = ext.values[r, ci]
    # base.columns already ends with the derived vram_usage_ratio: keep it last
    from ..viz.panels import VRAM_RATIO

    order = [c for c in cols if c != VRAM_RATIO] + extra + ([VRAM_RATIO] if VRAM_RATIO in cols else [])
    idx = [(cols + extra).index(c) for c in order]
    snap = NodeSnapshot(
        gpu_ids=list(base.gpu_ids),
        card_models=list(base.card_models),
        columns=tuple(order),
        values=vals[:, idx],
        power_limits=[ext.power_limits[r] if r >= 0 else None for r in rows],
        product_names=[(base.product_names[i] if i < len(base.product_names) and base.product_names[i] else "")
                       or (ext.product_names[r] if r >= 0 and r < len(ext.product_names) else "")
                       for i, r in enumerate(rows)],
        refresh_time=ext.refresh_time,
    )
    take = np.array([max(r, 0) for r in rows], dtype=np.int64)
    present = np.array([r >= 0 for r in rows])
    if ext.window is not None:
        w = ext.window[take].copy()
        w[~present] = np.nan
        last = STAT_INDEX["last"]
        for si, series in enumerate(ext.window_series):  # newest value: the merged columns
            if snap.has(series):
                w[:, si, last] = snap.values[:, snap.columns.index(series)]
        snap.window, snap.window_series = w, ext.window_series
    snap.node_window = ext.node_window
    if ext.node_window is not None and not snap.window_series:
        snap.window_series = ext.window_series
    if ext.xcd is not None:
        x = ext.xcd[take].copy()
        x[~present] = np.nan
        snap.xcd = x
    if ext.source_health is not None:
        h = ext.source_health.rows[take].copy()
        h[~present, :, HEALTH_INDEX["present"]] = 0.0
        snap.source_health = SourceHealth(h, [ext.source_health.backends[r] if r >= 0 else ("", "") for r in rows])
    return snap
