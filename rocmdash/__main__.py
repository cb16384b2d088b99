"""``python -m rocmdash <command> [args]``: one entry point for the tools.

    serve            rank-per-GPU node service (run under torchrun; /metrics, frames)
    exporter         single-process Prometheus exporter (synthetic / local GPUs)
    mock-prometheus  mock Prometheus /api/v1/query server (reference PromQL)
    record           capture a GPU's telemetry to .npz for replay
    build            compile the native runtime in-tree (hipcc, gfx950)
    doctor           check what the node service needs on this machine
"""

from __future__ import annotations

import sys

COMMANDS = {
    "serve": ("rocmdash.serve", "main"),
    "exporter": ("rocmdash.prom.exporter", "main"),
    "mock-prometheus": ("rocmdash.prom.mock", "main"),
    "record": ("rocmdash.runtime.record", "main"),
    "build": ("rocmdash._build", "main"),
    "doctor": ("rocmdash.doctor", "main"),
}


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    if not argv or argv[0] in ("-h", "--help") or argv[0] not in COMMANDS:
        print(__doc__.strip())
        return 0 if argv and argv[0] in ("-h", "--help") else 2
    import importlib

    mod, fn = COMMANDS[argv[0]]
    rc = getattr(importlib.import_module(mod), fn)(argv[1:])
    return int(rc or 0)


if __name__ == "__main__":
    raise SystemExit(main())
