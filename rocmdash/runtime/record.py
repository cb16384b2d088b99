"""Checkpoint / replay of telemetry streams.

``record`` snapshots the rings of a live ``GpuAgent`` (rows, timestamps and the GPU's
identity) into a small ``.npz``; a ``GpuAgent(source="replay", replay=path)`` then
feeds those rows back through native replay sources, so a capture of a real MI355X
drives the whole pipeline - rings, stats kernel, all-gather, frame - on any machine
(CPU tests use one recorded on the GPU box: tests/fixtures/). The files are plain
arrays plus a JSON string: loaded with ``allow_pickle=False``.

Reference counterpart: none (SURVEY.md §5 "Checkpoint / resume": optional ring
snapshot for replayable streams).

    python -m rocmdash.runtime.record --out capture.npz --seconds 10 [--device 0]
"""

from __future__ import annotations

import argparse
import json
import time

import numpy as np


def record(agent, path: str | None = None) -> dict:
    """Snapshot every ring of ``agent`` (newest window of rows, oldest first)."""
    out = {"info": dict(agent.info.as_dict())}
    out["info"]["series"] = list(out["info"]["series"])
    kinds = ["smi", "counter"]
    for kind, ring in zip(kinds, agent.rings):
        rows, ts = ring.window(ring.capacity)
        out[f"{kind}_rows"] = np.asarray(rows, dtype=np.float32)
        out[f"{kind}_ts"] = np.asarray(ts, dtype=np.uint64)
    if path:
        arrays = {k: v for k, v in out.items() if k != "info"}
        np.savez_compressed(path, info=np.array(json.dumps(out["info"])), **arrays)
    return out


def load_recording(path: str) -> dict:
    with np.load(path, allow_pickle=False) as z:
        rec = {k: z[k] for k in z.files if k != "info"}
        rec["info"] = json.loads(str(z["info"]))
    return upgrade_layout(rec)


def upgrade_layout(rec: dict) -> dict:
    """Map a recording's columns onto the current row layouts by series name: series
    added since the capture was made (e.g. the interconnect columns) replay as NaN -
    a failed read, which every statistic but ``last`` / ``count`` skips."""
    from ..models.schema import CTR_FIELDS, SMI_FIELDS

    names = list(rec.get("info", {}).get("series", []))
    start = 0
    for kind, fields in (("smi", SMI_FIELDS), ("counter", CTR_FIELDS)):
        rows = rec.get(f"{kind}_rows")
        if rows is None:
            continue
        width = rows.shape[1]
        recorded = names[start : start + width]
        start += width
        if tuple(recorded) == tuple(fields) or len(recorded) != width:
            continue
        out = np.full((rows.shape[0], len(fields)), np.nan, dtype=np.float32)
        for j, name in enumerate(recorded):
            if name in fields:
                out[:, fields.index(name)] = rows[:, j]
        rec[f"{kind}_rows"] = out
    if names:
        rec["info"]["series"] = list(SMI_FIELDS) + (list(CTR_FIELDS) if "counter_rows" in rec else [])
    return rec


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="record live telemetry of one GPU for replay")
    ap.add_argument("--out", required=True)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--smi-hz", type=float, default=100.0)
    ap.add_argument("--counter-hz", type=float, default=100.0)
    ap.add_argument("--load", action="store_true", help="run a bf16 GEMM loop meanwhile (busy GPU)")
    args = ap.parse_args(argv)
    from . import native

    native.load()
    native.enable_counters(only_device=args.device)
    import torch

    from ..config import SamplerConfig
    from .agent import GpuAgent

    cfg = SamplerConfig(smi_hz=args.smi_hz, counter_hz=args.counter_hz, window=2048, ring_capacity=8192)
    agent = GpuAgent(args.device, cfg=cfg)
    agent.start()
    t_end = time.time() + args.seconds
    if args.load:
        x = torch.randn(8192, 8192, device=f"cuda:{args.device}", dtype=torch.bfloat16)
        i = 0
        while time.time() < t_end:
            y = x @ x
            i += 1
            if i % 50 == 0:  # alternate busy and idle phases
                torch.cuda.synchronize()
                time.sleep(0.3)
        del y
        torch.cuda.synchronize()
    else:
        time.sleep(args.seconds)
    agent.stop()
    rec = record(agent, args.out)
    print(json.dumps({"out": args.out, "info": rec["info"],
                      **{k: list(v.shape) for k, v in rec.items() if k != "info"}}))
    agent.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
