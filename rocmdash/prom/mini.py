"""A small Prometheus: scrape loop, latest-value TSDB, ``/api/v1/query`` HTTP API.

Reference counterpart: the Prometheus server the reference talks to
(``PROMETHEUS_METRICS_ENDPOINT``, ``app.py:22``), which is external to it. This one
exists so the whole chain - exporter -> scrape -> instant query -> dashboard - runs
on one machine with no cluster: CPU tests (BASELINE.json config #1), the GPU-box
end-to-end check, and as a drop-in for a single-node deployment.

Semantics kept from Prometheus:
  * a scrape adds ``job`` and ``instance`` (``<host>:<port>`` of the target) labels,
    plus the synthetic ``up`` series;
  * an instant query at time t returns, per series, the newest sample in
    ``(t - lookback, t]`` (lookback 5 min) - stale series vanish;
  * the HTTP API's JSON envelope (``status`` / ``data.resultType`` = ``vector`` /
    ``result[].metric`` / ``result[].value = [unix_ts, "string"]``), which is exactly
    what the reference parses (``app.py:164, 183-188``).
"""

from __future__ import annotations

import json
import threading
import time
import urllib.parse
import urllib.request
from collections import OrderedDict
from dataclasses import dataclass, field
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from .exposition import format_value, parse_text
from .promql import Aggregate, PromQLError, aggregate, parse

LOOKBACK_S = 300.0


class TSDB:
    """Latest sample (and a short history) per series, keyed by the full label set and
    indexed by metric name: an instant query matches ``__name__`` against the distinct
    names first (a few dozen) and only then the label sets of the matching series, instead
    of every series of every GPU (thousands at 8 GPUs with window statistics)."""

    def __init__(self, history: int = 64):
        self._lock = threading.Lock()
        self._series: dict = {}  # key(tuple labels incl __name__) -> list[(ts, value)]
        self._by_name: dict = {}  # __name__ -> {key: (labels dict, hist, labels JSON, [ts, element])}
        self._mcache: dict = {}  # (label, op, value, label value) -> matched
        self.history = history

    def _hist(self, labels: dict, key: tuple) -> list:
        hist = self._series.get(key)
        if hist is None:
            hist = self._series[key] = []
            # the series' labels as API JSON, encoded once, and its newest result element
            # [ts, text] re-encoded only when a new sample arrives (query_json)
            self._by_name.setdefault(labels.get("__name__", ""), {})[key] = (dict(labels), hist, json.dumps(labels),
                                                                            [None, ""])
        return hist

    def add(self, labels: dict, value: float, ts: float | None = None) -> None:
        ts = time.time() if ts is None else ts
        key = tuple(sorted(labels.items()))
        with self._lock:
            hist = self._hist(labels, key)
            hist.append((ts, float(value)))
            if len(hist) > self.history:
                del hist[: len(hist) - self.history]

    def add_many(self, items, ts: float | None = None) -> None:
        ts = time.time() if ts is None else ts
        with self._lock:
            for labels, value in items:
                key = tuple(sorted(labels.items()))
                hist = self._hist(labels, key)
                hist.append((ts, float(value)))
                if len(hist) > self.history:
                    del hist[: len(hist) - self.history]

    def instant(self, selector, at: float | None = None, lookback: float = LOOKBACK_S) -> list:
        at = time.time() if at is None else at
        out = []
        with self._lock:
            for labels, ts, v, _, _ in self._matching(selector, at, lookback):
                out.append((dict(labels), v, ts))
        return out

    def instant_json(self, selector, at: float | None = None, lookback: float = LOOKBACK_S) -> list:
        """``instant`` as API JSON result elements (label JSON cached per series)."""
        at = time.time() if at is None else at
        out = []
        with self._lock:
            for _, ts, v, lj, cell in self._matching(selector, at, lookback):
                if cell[0] != (ts, v):
                    cell[0], cell[1] = (ts, v), '{"metric":%s,"value":[%r,"%s"]}' % (lj, ts, format_value(v))
                out.append(cell[1])
        return out

    def _match(self, m, value: str) -> bool:
        """A matcher against one label value, memoised (label values repeat across
        series and queries: instance, gpu_id, stat ...)."""
        k = (m.label, m.op, m.value, value)
        hit = self._mcache.get(k)
        if hit is None:
            if len(self._mcache) > 100_000:
                self._mcache.clear()
            hit = self._mcache[k] = m.matches(value)
        return hit

    def _matching(self, selector, at: float, lookback: float):
        """(labels, ts, value, labels JSON, cached element) of the newest sample at or
        before ``at`` (within ``lookback``) of every series the selector matches; caller
        holds the lock."""
        name_ms = [m for m in selector.matchers if m.label == "__name__"]
        others = [m for m in selector.matchers if m.label != "__name__"]
        for name, group in self._by_name.items():
            if not all(self._match(m, name) for m in name_ms):
                continue
            for labels, hist, lj, cell in group.values():
                if not all(self._match(m, labels.get(m.label, "")) for m in others):
                    continue
                for ts, v in reversed(hist):
                    if ts <= at:
                        if ts > at - lookback:
                            yield labels, ts, v, lj, cell
                        break

    def series_count(self) -> int:
        with self._lock:
            return len(self._series)

    def clear(self) -> None:
        with self._lock:
            self._series.clear()
            self._by_name.clear()
            self._mcache.clear()


@dataclass
class Target:
    url: str  # http://host:port/metrics
    job: str = "amd-gpu-exporter"
    instance: str = ""
    extra_labels: dict = field(default_factory=dict)
    last_error: str = ""
    last_scrape_s: float = 0.0
    health: str = "unknown"

    def __post_init__(self):
        if not self.instance:
            u = urllib.parse.urlparse(self.url)
            self.instance = u.netloc


class MiniPrometheus:
    def __init__(self, scrape_interval: float = 1.0, timeout: float = 2.0):
        self.db = TSDB()
        self.targets: list = []
        self.scrape_interval = scrape_interval
        self.timeout = timeout
        self._stop = threading.Event()
        self._thread = None
        self._server = None
        self.queries = 0
        # query text -> parsed expression, bounded LRU: the page sends the same three
        # queries every refresh, an ad-hoc client never evicts them for long
        self._parsed: OrderedDict = OrderedDict()
        self._parsed_lock = threading.Lock()

    # ----------------------------------------------------------------- scraping
    def add_target(self, url: str, **kw) -> Target:
        t = Target(url, **kw)
        self.targets.append(t)
        return t

    def scrape_once(self, target: Target, at: float | None = None) -> bool:
        at = time.time() if at is None else at
        t0 = time.perf_counter()
        up = 0.0
        try:
            with urllib.request.urlopen(target.url, timeout=self.timeout) as r:
                text = r.read().decode("utf-8")
            base = {"job": target.job, "instance": target.instance}
            base.update(target.extra_labels)
            items = []
            for s in parse_text(text):
                labels = dict(s.labels)
                # honor_labels=false: target labels win over exported ones
                for k, v in base.items():
                    if k in labels:
                        labels["exported_" + k] = labels[k]
                    labels[k] = v
                labels["__name__"] = s.name
                items.append((labels, s.value))
            self.db.add_many(items, at)
            up = 1.0
            target.health = "up"
            target.last_error = ""
        except Exception as exc:  # a down target is data ("up" = 0), not a crash
            target.health = "down"
            target.last_error = str(exc)
        target.last_scrape_s = time.perf_counter() - t0
        self.db.add({"__name__": "up", "job": target.job, "instance": target.instance}, up, at)
        return up == 1.0

    def scrape_all(self) -> None:
        for t in self.targets:
            self.scrape_once(t)

    def start_scraping(self) -> None:
        if self._thread is not None:
            return

        def loop():
            while not self._stop.is_set():
                t0 = time.monotonic()
                self.scrape_all()
                self._stop.wait(max(0.0, self.scrape_interval - (time.monotonic() - t0)))

        self._thread = threading.Thread(target=loop, name="mini-prom-scrape", daemon=True)
        self._thread.start()

    # ----------------------------------------------------------------- queries
    _PARSED_MAX = 256

    def _expr(self, q: str):
        """The parsed expression of ``q`` (raises PromQLError on bad PromQL), from the
        LRU cache; parsed at most once per cache residency."""
        with self._parsed_lock:
            expr = self._parsed.get(q)
            if expr is not None:
                self._parsed.move_to_end(q)
                return expr
        expr = parse(q)
        with self._parsed_lock:
            self._parsed[q] = expr
            while len(self._parsed) > self._PARSED_MAX:
                self._parsed.popitem(last=False)
        return expr

    def query(self, q: str, at: float | None = None) -> dict:
        """Evaluate an instant query; returns the API's ``data`` object."""
        self.queries += 1
        return self._evaluate(self._expr(q), at)

    def _evaluate(self, expr, at: float | None) -> dict:
        at = time.time() if at is None else at
        if isinstance(expr, Aggregate):
            rows = [(labels, v) for labels, v, _ in self.db.instant(expr.selector, at)]
            res = [
                {"metric": labels, "value": [at, format_value(v)]}
                for labels, v in aggregate(expr, rows)
            ]
        else:
            res = [{"metric": labels, "value": [ts, format_value(v)]} for labels, v, ts in self.db.instant(expr, at)]
        return {"resultType": "vector", "result": res}

    def query_json(self, q: str, at: float | None = None) -> str:
        """The whole API response of an instant query as JSON text. Selector queries are
        assembled from each series' cached label JSON (the page's queries return ~150
        series per GPU); aggregates go through ``query``."""
        expr = self._expr(q)  # parsed once; PromQLError for bad PromQL
        self.queries += 1
        if isinstance(expr, Aggregate):
            return json.dumps({"status": "success", "data": self._evaluate(expr, at)})
        res = self.db.instant_json(expr, at)
        return '{"status":"success","data":{"resultType":"vector","result":[' + ",".join(res) + "]}}"

    # ----------------------------------------------------------------- HTTP
    def serve(self, host: str = "127.0.0.1", port: int = 9090) -> ThreadingHTTPServer:
        prom = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"
            # headers and body leave in two writes: without TCP_NODELAY the body waits for
            # the client's delayed ACK of the headers (~40 ms per keep-alive request)
            disable_nagle_algorithm = True

            def log_message(self, *a):  # quiet
                pass

            def _send(self, code: int, obj=None, text: str | None = None, ctype="application/json"):
                body = (text if text is not None else json.dumps(obj)).encode()
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _params(self):
                u = urllib.parse.urlparse(self.path)
                params = dict(urllib.parse.parse_qsl(u.query))
                if self.command == "POST":
                    n = int(self.headers.get("Content-Length", "0") or 0)
                    if n:
                        params.update(urllib.parse.parse_qsl(self.rfile.read(n).decode()))
                return u.path, params

            def _handle(self):
                path, params = self._params()
                if path == "/api/v1/query":
                    q = params.get("query")
                    if not q:
                        return self._send(400, {"status": "error", "errorType": "bad_data", "error": "missing query"})
                    try:
                        at = float(params["time"]) if "time" in params else None
                        body = prom.query_json(q, at)  # one parse (cached) + one evaluation
                    except (PromQLError, ValueError) as exc:
                        return self._send(400, {"status": "error", "errorType": "bad_data", "error": str(exc)})
                    return self._send(200, text=body)
                if path == "/api/v1/targets":
                    act = [
                        {
                            "scrapeUrl": t.url,
                            "labels": {"job": t.job, "instance": t.instance},
                            "health": t.health,
                            "lastError": t.last_error,
                            "lastScrapeDuration": t.last_scrape_s,
                        }
                        for t in prom.targets
                    ]
                    return self._send(200, {"status": "success", "data": {"activeTargets": act}})
                if path in ("/-/healthy", "/-/ready"):
                    return self._send(200, text="OK\n", ctype="text/plain")
                return self._send(404, {"status": "error", "error": "not found"})

            do_GET = _handle
            do_POST = _handle

        srv = ThreadingHTTPServer((host, port), Handler)
        srv.daemon_threads = True
        th = threading.Thread(target=srv.serve_forever, name="mini-prom-http", daemon=True)
        th.start()
        self._server = srv
        return srv

    @property
    def port(self) -> int:
        return self._server.server_address[1] if self._server else 0

    def close(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None
        if self._server is not None:
            self._server.shutdown()
            self._server.server_close()
            self._server = None
