"""Prometheus text exposition (format 0.0.4): render and parse.

The exporter publishes the series the reference dashboard queries
(``app.py:168-171``: ``amd_gpu_edge_temperature``, ``amd_gpu_gfx_activity``,
``amd_gpu_average_package_power``, ``amd_gpu_used_vram``, ``amd_gpu_total_vram``)
with the labels it reads (``gpu_id``, ``card_model``, ``app.py:186-192``); Prometheus
adds ``instance=<node-ip>:<port>`` at scrape time, which the reference's second
query filters on (``app.py:171``). New series: the other amd-smi / counter columns,
the window statistics of every series (``rocmdash_window{metric,stat}``) and the
exporter's own health metrics.

Rendering is plain string building (no client-library registry) so one scrape of an
8-GPU node costs tens of microseconds; ``parse_text`` is the matching parser used by
the mini-Prometheus scraper. Both are checked against ``prometheus_client``'s parser
in tests/test_prom.py.
"""

from __future__ import annotations

import math
import re
from typing import NamedTuple

from ..models.schema import METRIC_SPECS, STAT_NAMES


def escape_label_value(v) -> str:
    return str(v).replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


def format_value(v) -> str:
    if v is None:
        return "NaN"
    v = float(v)
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    if v == int(v) and abs(v) < 1e15:
        return str(int(v))
    return repr(v)


def _labels(d: dict) -> str:
    if not d:
        return ""
    return "{" + ",".join(f'{k}="{escape_label_value(v)}"' for k, v in d.items()) + "}"


class Exposition:
    """Accumulates families; ``text()`` renders HELP/TYPE once per family."""

    def __init__(self):
        self._fams: dict = {}

    def add(self, name: str, value, labels: dict | None = None, help: str = "", typ: str = "gauge",
            family: str | None = None) -> None:
        """Add one sample. ``family`` groups suffixed samples (``x_bucket``, ``x_sum``,
        ``x_count`` of histogram ``x``) under one HELP/TYPE header."""
        fam_name = family or name
        fam = self._fams.get(fam_name)
        if fam is None:
            fam = self._fams[fam_name] = (help, typ, [])
        fam[2].append((name, labels or {}, value))

    def text(self) -> str:
        out = []
        for fam_name, (help_, typ, samples) in self._fams.items():
            if help_:
                out.append(f"# HELP {fam_name} {help_.replace(chr(92), chr(92) * 2).replace(chr(10), chr(92) + 'n')}")
            out.append(f"# TYPE {fam_name} {typ}")
            for name, labels, value in samples:
                out.append(f"{name}{_labels(labels)} {format_value(value)}")
        return "\n".join(out) + "\n"


def render_snapshot(snap, hostname: str = "", extra_labels: dict | None = None, window_stats=("p50", "p90", "p99", "min", "max", "mean")) -> str:
    """Exposition for a ``NodeSnapshot`` (latest values + window statistics)."""
    exp = Exposition()
    extra = dict(extra_labels or {})
    for g, gid in enumerate(snap.gpu_ids):
        base = {"gpu_id": gid, "card_model": snap.card_models[g] or ""}
        if hostname:
            base["hostname"] = hostname
        base.update(extra)
        for c, col in enumerate(snap.columns):
            if col == "vram_usage_ratio":
                continue
            spec = METRIC_SPECS.get(col)
            exp.add(col, snap.values[g, c], base, spec.help + f" ({spec.unit})" if spec else "")
        pl = snap.power_limits[g] if g < len(snap.power_limits) else None
        if pl:
            exp.add("amd_gpu_power_cap", pl, base, "Socket power cap reported by amd-smi (W)")
        pn = snap.product_names[g] if g < len(snap.product_names) else None
        if pn:  # lets a reader name a board whose part number it does not know
            exp.add("amd_gpu_info", 1, dict(base, product_name=pn), "Board identity reported by amd-smi (value 1)")
    if snap.window is not None and len(snap.window_series):
        idx = [(s, STAT_NAMES.index(s)) for s in window_stats]
        for g, gid in enumerate(snap.gpu_ids):
            base = {"gpu_id": gid, "card_model": snap.card_models[g] or ""}
            if hostname:
                base["hostname"] = hostname
            base.update(extra)
            for si, series in enumerate(snap.window_series):
                for sname, k in idx:
                    lab = dict(base)
                    lab["metric"] = series
                    lab["stat"] = sname
                    exp.add("rocmdash_window", snap.window[g, si, k], lab, "Window statistic of a series over the last W samples (HIP window-stats kernel)")
                lab = dict(base)
                lab["metric"] = series
                exp.add("rocmdash_window_samples", snap.window[g, si, STAT_NAMES.index("count")], lab, "Valid samples in the statistics window")
    xcd = getattr(snap, "xcd", None)
    if xcd is not None:
        for g, gid in enumerate(snap.gpu_ids):
            base = {"gpu_id": gid, "card_model": snap.card_models[g] or ""}
            if hostname:
                base["hostname"] = hostname
            base.update(extra)
            for x in range(xcd.shape[2]):
                if math.isnan(float(xcd[g, 0, x])) and math.isnan(float(xcd[g, 1, x])):
                    continue  # no such XCD on this part / mode
                lab = dict(base)
                lab["xcd"] = str(x)
                exp.add("amd_gpu_xcd_activity", xcd[g, 0, x], lab, "Busy of one accelerator complex die (XCD) (%)")
                exp.add("amd_gpu_xcd_gfx_clock", xcd[g, 1, x], lab, "Current gfx clock of one XCD (MHz)")
    health = getattr(snap, "source_health", None)
    if health is not None:
        render_health(exp, health, snap.gpu_ids, hostname, extra)
    if snap.node_window is not None and len(snap.window_series):
        base = {"hostname": hostname} if hostname else {}
        base.update(extra)
        for si, series in enumerate(snap.window_series):
            for sname in tuple(window_stats) + ("count",):
                lab = dict(base)
                lab["metric"] = series
                lab["stat"] = sname
                exp.add("rocmdash_node_window", snap.node_window[si, STAT_NAMES.index(sname)], lab,
                        "Window statistic of a series over every GPU's window at once (node-wide)")
    return exp.text()


def render_health(exp: Exposition, health, gpu_ids, hostname: str = "", extra: dict | None = None) -> None:
    """Sampler health of every source of every GPU (``rocmdash.models.health``)."""
    for st in health.statuses():
        lab = {"gpu_id": gpu_ids[st.gpu], "source": st.kind, "backend": st.backend}
        if hostname:
            lab["hostname"] = hostname
        lab.update(extra or {})
        exp.add("rocmdash_sampler_samples_total", st.samples, lab, "Rows pushed into the ring", "counter")
        exp.add("rocmdash_sampler_failures_total", st.failures, lab, "Failed source reads", "counter")
        exp.add("rocmdash_sampler_overruns_total", st.overruns, lab, "Missed sampling deadlines", "counter")
        exp.add("rocmdash_sample_age_seconds", st.age_s, lab, "Age of the newest sample (staleness)")
        exp.add("rocmdash_sampler_rate_hz", st.hz, lab, "Configured sampling rate of the source")
        exp.add("rocmdash_source_stale", 1.0 if st.stale else 0.0, lab,
                "1 if the source produced no sample within stale_periods periods")


# ----------------------------------------------------------------------------- parse
class Sample(NamedTuple):
    name: str
    labels: tuple  # sorted ((k, v), ...)
    value: float
    timestamp_ms: int | None = None

    def label_dict(self) -> dict:
        return dict(self.labels)


_NAME = r"[a-zA-Z_:][a-zA-Z0-9_:]*"
_LINE = re.compile(rf"^({_NAME})(?:\{{(.*)\}})?\s+(\S+)(?:\s+(-?\d+))?\s*$")
_LABEL = re.compile(r'\s*([a-zA-Z_][a-zA-Z0-9_]*)\s*=\s*"((?:[^"\\]|\\.)*)"\s*,?')


def _unescape(s: str) -> str:
    if "\\" not in s:
        return s
    out = []
    i = 0
    while i < len(s):
        c = s[i]
        if c == "\\" and i + 1 < len(s):
            n = s[i + 1]
            out.append("\n" if n == "n" else n)
            i += 2
        else:
            out.append(c)
            i += 1
    return "".join(out)


def parse_value(s: str) -> float:
    try:
        return float(s)  # accepts nan / inf / +inf / -inf in any case as well
    except ValueError:
        pass
    s = s.strip()
    low = s.lower()
    if low in ("nan",):
        return float("nan")
    if low in ("+inf", "inf"):
        return float("inf")
    if low == "-inf":
        return float("-inf")
    return float(s)


def _parse_labels(lab: str, line: str) -> tuple:
    pairs = []
    pos = 0
    while pos < len(lab):
        lm = _LABEL.match(lab, pos)
        if not lm:
            if lab[pos:].strip() == "":
                break
            raise ValueError(f"bad labels in line: {line!r}")
        pairs.append((lm.group(1), _unescape(lm.group(2))))
        pos = lm.end()
    return tuple(sorted(pairs))


# label blocks repeat exactly from one scrape of a target to the next: parsed once
_LABEL_CACHE: dict = {}
_LABEL_CACHE_MAX = 16384


def parse_text(text: str) -> list:
    """Parse exposition text into ``Sample``s (comments/HELP/TYPE skipped)."""
    out = []
    cache = _LABEL_CACHE
    # "\n" is the only line separator of the format: str.splitlines() would also split
    # inside label values at \x1c-\x1e, \x85, \u2028 ... (found by tests/test_properties.py)
    for line in text.split("\n"):
        line = line.rstrip("\r")
        if not line or line[0] == "#":
            continue
        m = _LINE.match(line)
        if not m:
            raise ValueError(f"bad exposition line: {line!r}")
        name, lab, val, ts = m.groups()
        labels = ()
        if lab:
            labels = cache.get(lab)
            if labels is None:
                labels = _parse_labels(lab, line)
                if len(cache) >= _LABEL_CACHE_MAX:
                    cache.clear()
                cache[lab] = labels
        out.append(Sample(name, labels, parse_value(val), int(ts) if ts else None))
    return out
