"""Prometheus query layer with the reference's contract.

Reference: ``fetch_gpu_metrics`` (``app.py:153-227``):
  1. node discovery: ``kube_pod_info{pod=~".*<PODNAME>.*"}`` -> ``host_ip`` of the
     FIRST result (``app.py:157-164``);
  2. one instant query for the five ``amd_gpu_*`` series on ``instance=~"<ip>:.+"``
     (``app.py:167-178``);
  3. long rows -> ``pivot(index='gpu_id', columns='metric_name')`` + ``card_model``
     (first seen per GPU) -> ``vram_usage_ratio`` -> mean/max/min stats over all GPUs
     (``app.py:180-221``);
  4. any exception -> error banner + ``(None, None)`` (``app.py:225-227``).

Kept: both PromQL strings byte for byte, the env vars and defaults, the return
shapes, the error path for duplicate (gpu, metric) series and for a missing
``amd_gpu_total_vram`` / ``amd_gpu_used_vram`` column. Changed:
requests carry a timeout and reuse one keep-alive connection, metric columns are float64 and
the long->wide step builds the table directly instead of through ``DataFrame.pivot``.

``fetch_node_snapshot`` is the fast form used by the app: it returns a
``NodeSnapshot`` and never touches pandas.
"""

from __future__ import annotations

import logging
import math
import os

from .. import config
from ..models.schema import COMPAT_METRICS
from ..viz.panels import NodeSnapshot

log = logging.getLogger("rocmdash.prom.query")


def node_discovery_query(podname: str | None = None) -> str:
    """``app.py:157``."""
    pod = config.PROMETHEUS_METRICS_PODNAME if podname is None else podname
    return f"kube_pod_info{{pod=~\".*{pod}.*\"}}"


def gpu_metrics_query(node_ip: str, metrics=COMPAT_METRICS) -> str:
    """``app.py:167-172`` (same string for the default metric set)."""
    return "{__name__=~\"" + "|".join(metrics) + "\", instance=~\"" + node_ip + ":.+\"}"


class QueryError(RuntimeError):
    pass


class HTTPStatusError(OSError):
    """Non-2xx answer from Prometheus (``raise_for_status``, ``app.py:162, 177``)."""


class _Response:
    __slots__ = ("status_code", "content", "reason")

    def __init__(self, status: int, content: bytes, reason: str):
        self.status_code, self.content, self.reason = status, content, reason

    @property
    def text(self) -> str:
        return self.content.decode("utf-8", "replace")

    def json(self):
        import json

        return json.loads(self.content)

    def raise_for_status(self) -> None:
        if self.status_code >= 400:
            raise HTTPStatusError(f"{self.status_code} {self.reason}")


class KeepAliveGet:
    """``requests.get``-shaped GET over ONE persistent HTTP/1.1 connection (stdlib
    ``http.client``): the page's three instant queries per refresh reuse it. requests'
    session machinery (adapters, hooks, cookie jars, header merging) cost more than the
    query itself on the page path (tools/probes/probe_page_client.py). A dropped
    keep-alive connection is reopened once per call. One connection per calling thread
    (Streamlit runs every browser session on its own thread)."""

    def __init__(self):
        import threading

        self._tls = threading.local()

    def __call__(self, url: str, params: dict | None = None, timeout: float | None = None):
        import http.client
        from urllib.parse import urlencode, urlsplit

        u = urlsplit(url)
        key = (u.scheme, u.hostname, u.port, timeout)
        path = (u.path or "/") + ("?" + urlencode(params) if params else "")
        tls = self._tls
        for attempt in (0, 1):
            if getattr(tls, "conn", None) is None or tls.key != key:
                self.close()
                cls = http.client.HTTPSConnection if u.scheme == "https" else http.client.HTTPConnection
                tls.conn = cls(u.hostname, u.port, timeout=timeout)
                tls.key = key
            try:
                tls.conn.request("GET", path, headers={"Accept": "application/json", "Connection": "keep-alive"})
                r = tls.conn.getresponse()
                body = r.read()
                if r.getheader("Connection", "").lower() == "close":
                    self.close()
                return _Response(r.status, body, r.reason)
            except (http.client.HTTPException, ConnectionError, BrokenPipeError):
                self.close()
                if attempt:
                    raise

    def close(self) -> None:
        """Close the calling thread's connection."""
        conn = getattr(self._tls, "conn", None)
        if conn is not None:
            conn.close()
            self._tls.conn = None


class PrometheusClient:
    """Thin HTTP client for ``/api/v1/query`` with a persistent connection + timeout.

    ``get`` may be injected (tests and the CPU benchmark pass a fake with the
    ``requests.get`` signature); the default is ``KeepAliveGet``."""

    def __init__(self, endpoint: str | None = None, timeout: float | None = None, get=None):
        self.endpoint = endpoint or config.PROMETHEUS_METRICS_ENDPOINT
        self.timeout = config.HTTP_TIMEOUT_S if timeout is None else timeout
        self._get = get
        self._session = None

    def _http_get(self):
        if self._get is not None:
            return self._get
        if self._session is None:
            # behind an HTTP(S) proxy the reference's requests session (which honours the
            # proxy environment) is kept; otherwise one plain keep-alive connection
            if any(os.environ.get(k) for k in ("HTTP_PROXY", "HTTPS_PROXY", "http_proxy", "https_proxy")):
                import requests

                self._session = requests.Session()
            else:
                self._session = KeepAliveGet()
        return self._session.get if hasattr(self._session, "get") else self._session

    def query(self, promql: str) -> list:
        resp = self._http_get()(url=self.endpoint, params={"query": promql}, timeout=self.timeout)
        resp.raise_for_status()
        body = resp.json() if hasattr(resp, "json") else None
        if body is None:
            import json

            body = json.loads(resp.text)
        if body.get("status") not in (None, "success"):
            raise QueryError(f"Prometheus error: {body.get('errorType')}: {body.get('error')}")
        return body["data"]["result"]

    def node_ip(self, podname: str | None = None) -> str:
        res = self.query(node_discovery_query(podname))
        return res[0]["metric"]["host_ip"]  # first match only, like app.py:164

    def close(self):
        if self._session is not None:
            self._session.close()
            self._session = None


def _long_to_wide(result, metrics_required=("amd_gpu_used_vram", "amd_gpu_total_vram")):
    """Parse instant-vector results into (gpu_ids, card_models, columns, rows).

    Raises like the reference's pivot: duplicate (gpu_id, metric) -> ValueError;
    a missing used/total VRAM column -> KeyError."""
    table: dict = {}
    models: dict = {}
    names: dict = {}
    for item in result:
        m = item["metric"]
        gid = m["gpu_id"]
        name = m["__name__"]
        val = float(item["value"][1])
        row = table.get(gid)
        if row is None:
            row = table[gid] = {}
        if name in row:
            raise ValueError("Index contains duplicate entries, cannot reshape")
        row[name] = val
        names[name] = None
        if gid not in models:
            models[gid] = m["card_model"]
    for req in metrics_required:
        if req not in names:
            raise KeyError(req)
    columns = tuple(sorted(names))
    gpu_ids = sorted(table)  # pivot sorts its index (lexicographic on strings)
    rows = [[table[g].get(c, math.nan) for c in columns] for g in gpu_ids]
    return gpu_ids, [models[g] for g in gpu_ids], columns, rows


def extended_enabled() -> bool:
    return os.environ.get("ROCMDASH_EXTENDED", "0") not in ("0", "", "false", "off")


def fetch_node_snapshot(client: PrometheusClient | None = None, podname: str | None = None, metrics=COMPAT_METRICS,
                        extended: bool | None = None) -> NodeSnapshot:
    """Discovery + metric query -> ``NodeSnapshot`` (raises on any failure).

    ``extended`` (default ``ROCMDASH_EXTENDED``): after the reference's two queries,
    ONE more instant query on the same node fetches what the node service exports
    beyond the five compat series - MFMA / HBM / xGMI / PCIe columns, the window
    statistics of every series, node-wide window statistics, per-XCD detail and every
    GPU's sampler health (``snapshot_io.extended_query``) - and widens the snapshot
    with it. The compat query, its GPU set and its error paths are unchanged."""
    client = client or PrometheusClient()
    ip = client.node_ip(podname)
    result = client.query(gpu_metrics_query(ip, metrics))
    gpu_ids, models, columns, rows = _long_to_wide(result)
    snap = NodeSnapshot(gpu_ids=gpu_ids, card_models=models, columns=columns, values=rows)
    if extended if extended is not None else extended_enabled():
        from .snapshot_io import extended_query, merge_extended, snapshot_from_series

        ext = client.query(extended_query(ip))
        items = ((dict(r["metric"]), r["value"][1]) for r in ext)
        snap = merge_extended(snap, snapshot_from_series(items, require_vram=False))
    return snap


_SERVICE_GET = None


def fetch_service_snapshot(url: str | None = None, timeout: float | None = None, get=None) -> NodeSnapshot:
    """One scrape of the rank-per-GPU node service's ``/metrics`` (``rocmdash.serve``,
    rank 0) -> ``NodeSnapshot``: the RCCL-gathered node tensor with every series,
    window statistics, node-window statistics, per-XCD detail and per-rank source
    health, no Prometheus in between (the page's ``native`` data source)."""
    from .exposition import parse_text
    from .snapshot_io import snapshot_from_series

    url = url or os.environ.get("ROCMDASH_NODE_ENDPOINT", "http://127.0.0.1:%d/metrics" % config.EXPORTER_PORT)
    if get is None:
        global _SERVICE_GET
        if any(os.environ.get(k) for k in ("HTTP_PROXY", "HTTPS_PROXY", "http_proxy", "https_proxy")):
            import requests

            get = requests.get
        else:  # one keep-alive connection for the page's refreshes (KeepAliveGet)
            if _SERVICE_GET is None:
                _SERVICE_GET = KeepAliveGet()
            get = _SERVICE_GET
    resp = get(url, timeout=config.HTTP_TIMEOUT_S if timeout is None else timeout)
    resp.raise_for_status()
    items = ((dict(s.labels, __name__=s.name), s.value) for s in parse_text(resp.text))
    return snapshot_from_series(items)


def _default_error(msg: str) -> None:
    try:  # the reference reports through a Streamlit banner (app.py:226)
        import streamlit as st

        st.error(msg)
    except Exception:
        log.error(msg)


def fetch_gpu_metrics(client: PrometheusClient | None = None, on_error=None):
    """Reference-compatible ``fetch_gpu_metrics() -> (df_pivot, stats) | (None, None)``."""
    try:
        snap = fetch_node_snapshot(client, extended=False)  # the reference's columns only
        return snap.to_dataframe()
    except Exception as e:  # same catch-all as app.py:225
        (on_error or _default_error)(f"Error fetching GPU metrics: {str(e)}")
        return None, None
