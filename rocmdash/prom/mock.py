"""Synthetic node for the Prometheus path (BASELINE.json config #1: the dashboard on
a CPU reading synthetic Prometheus JSON, no GPU).

``SyntheticNode`` produces what a real deployment's Prometheus would hold for one
node: the exporter's ``amd_gpu_*`` series per GPU with ``gpu_id`` / ``card_model``
labels on ``instance=<host_ip>:<port>`` (``app.py:168-171, 186-192``) and
kube-state-metrics' ``kube_pod_info{pod, host_ip}`` for the Prometheus pod
(``app.py:157-164``). ``prometheus_response`` renders the ``/api/v1/query`` JSON
directly (for monkeypatched HTTP in tests and the CPU benchmark); ``MockPrometheus``
serves it over HTTP through ``MiniPrometheus``.

    python -m rocmdash.prom.mock --gpus 8 --port 9090
"""

from __future__ import annotations

import argparse
import json
import random
import time

from ..models.schema import COMPAT_METRICS
from .exposition import format_value
from .mini import MiniPrometheus

MI355X_PART = "102-G36236-0C"
MI300_PART = "102-G30211-0C"


class SyntheticNode:
    def __init__(
        self,
        n_gpus: int = 8,
        host_ip: str = "10.0.0.5",
        exporter_port: int = 5000,
        card_model: str = MI355X_PART,
        pod: str = "prometheus-server-0",
        seed: int = 0,
        total_vram_mb: float = 294896.0,
        gpu_ids=None,
        extra_metrics=(),
    ):
        self.n = n_gpus
        self.host_ip = host_ip
        self.port = exporter_port
        self.card_model = card_model
        self.pod = pod
        self.rng = random.Random(seed)
        self.total = total_vram_mb
        self.gpu_ids = [str(g) for g in (gpu_ids if gpu_ids is not None else range(n_gpus))]
        self.extra_metrics = tuple(extra_metrics)
        self.t = 0
        self.state = [
            {"util": self.rng.uniform(20, 95), "temp": self.rng.uniform(40, 70), "used": self.rng.uniform(0.1, 0.9)}
            for _ in self.gpu_ids
        ]
        self.overrides: dict = {}  # (gpu_id, metric) -> value (fault injection / fixtures)
        self.drop: set = set()  # (gpu_id, metric) pairs to omit
        self.duplicate: set = set()  # (gpu_id, metric) pairs to emit twice (second exporter port)

    def step(self) -> None:
        self.t += 1
        for s in self.state:
            s["util"] = min(100.0, max(0.0, s["util"] + self.rng.gauss(0, 4)))
            s["temp"] += 0.05 * (35 + 0.4 * s["util"] - s["temp"]) + self.rng.gauss(0, 0.3)
            s["used"] = min(0.99, max(0.01, s["used"] + self.rng.gauss(0, 0.01)))

    def values(self, gpu_index: int) -> dict:
        s = self.state[gpu_index]
        power = 150 + 10.5 * s["util"]
        v = {
            "amd_gpu_edge_temperature": round(s["temp"]),
            "amd_gpu_gfx_activity": round(s["util"]),
            "amd_gpu_average_package_power": round(power),
            "amd_gpu_used_vram": round(s["used"] * self.total),
            "amd_gpu_total_vram": self.total,
        }
        for m in self.extra_metrics:
            v[m] = round(self.rng.uniform(0, 100), 2)
        return v

    def series(self):
        """[(labels, value)] for every series this node exports, plus kube_pod_info."""
        out = [
            (
                {
                    "__name__": "kube_pod_info",
                    "pod": self.pod,
                    "namespace": "monitoring",
                    "host_ip": self.host_ip,
                    "node": "mi355x-node-0",
                    "job": "kube-state-metrics",
                    "instance": "10.96.0.20:8080",
                },
                1.0,
            )
        ]
        inst = f"{self.host_ip}:{self.port}"
        for g, gid in enumerate(self.gpu_ids):
            for name, val in self.values(g).items():
                if (gid, name) in self.drop:
                    continue
                val = self.overrides.get((gid, name), val)
                labels = {
                    "__name__": name,
                    "gpu_id": gid,
                    "card_model": self.card_model,
                    "hostname": "mi355x-node-0",
                    "instance": inst,
                    "job": "amd-gpu-exporter",
                }
                out.append((labels, val))
                if (gid, name) in self.duplicate:
                    dup = dict(labels)
                    dup["instance"] = f"{self.host_ip}:{self.port + 1}"
                    out.append((dup, val))
        return out

    def populate(self, prom: MiniPrometheus, at: float | None = None) -> None:
        prom.db.add_many(self.series(), at)


def prometheus_response(result) -> str:
    """``/api/v1/query`` JSON for [(labels, value)] (what Prometheus returns)."""
    ts = time.time()
    return json.dumps(
        {
            "status": "success",
            "data": {
                "resultType": "vector",
                "result": [{"metric": labels, "value": [ts, format_value(v)]} for labels, v in result],
            },
        }
    )


class FakeResponse:
    """Minimal ``requests.Response`` stand-in (``.text``, ``.json()``,
    ``.status_code``, ``.raise_for_status()``)."""

    def __init__(self, text: str, status_code: int = 200):
        self.text = text
        self.status_code = status_code
        self.content = text.encode()

    def json(self):
        return json.loads(self.text)

    def raise_for_status(self):
        if self.status_code >= 400:
            import requests

            raise requests.HTTPError(f"{self.status_code} Server Error", response=self)


class FakePrometheusHTTP:
    """Callable replacing ``requests.get``/``Session.get``: evaluates the query against
    a ``SyntheticNode`` through the real PromQL engine, no sockets."""

    def __init__(self, node: SyntheticNode, status_code: int = 200, body: str | None = None):
        self.node = node
        self.prom = MiniPrometheus()
        self.status_code = status_code
        self.body = body
        self.calls = 0

    def __call__(self, url=None, params=None, timeout=None, **kw):
        self.calls += 1
        if self.status_code != 200 or self.body is not None:
            return FakeResponse(self.body if self.body is not None else "{}", self.status_code)
        self.prom.db.clear()
        self.node.populate(self.prom)
        q = (params or {}).get("query", "")
        data = self.prom.query(q)
        return FakeResponse(json.dumps({"status": "success", "data": data}))


class MockPrometheus(MiniPrometheus):
    """HTTP mock Prometheus backed by a synthetic node that advances every query."""

    def __init__(self, node: SyntheticNode | None = None, advance: bool = True):
        super().__init__()
        self.node = node or SyntheticNode()
        self.advance = advance
        self.node.populate(self)

    def query(self, q: str, at=None) -> dict:
        if self.advance:
            self.node.step()
        self.node.populate(self)
        return super().query(q, at)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Mock Prometheus serving a synthetic MI355X node")
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9090)
    ap.add_argument("--host-ip", default="10.0.0.5")
    ap.add_argument("--card-model", default=MI355X_PART)
    args = ap.parse_args(argv)
    mp = MockPrometheus(SyntheticNode(args.gpus, host_ip=args.host_ip, card_model=args.card_model))
    mp.serve(args.host, args.port)
    print(f"mock Prometheus on http://{args.host}:{mp.port}/api/v1/query ({args.gpus} GPUs)", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        mp.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

__all__ = ["COMPAT_METRICS", "FakePrometheusHTTP", "FakeResponse", "MockPrometheus", "SyntheticNode", "prometheus_response"]
