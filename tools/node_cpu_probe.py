"""Node-total CPU of the supervised service at production rates.

Starts ``python -m rocmdash.launch --nproc N ... -m rocmdash.serve`` (the DaemonSet's
entrypoint: amd-smi 10 Hz, device counters 100 Hz, 1 Hz node refresh), waits until every
GPU is on /metrics with fresh counter rows, then reads the supervisor's
``rocmdash_node_cpu_seconds_total{process}`` twice ``--seconds`` apart and every GPU's
counter-row count (``rocmdash_sampler_samples_total{source="counter"}``). One JSON line:
node CPU-s/s by process kind and in total, and each GPU's counter rows per second.

    ROCMDASH_OVERSUBSCRIBE=1 python tools/node_cpu_probe.py --nproc 8 --counter-daemon on
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def read(port):
    from _supervisor_helpers import get

    from rocmdash.prom.exposition import parse_text

    code, body = get(f"http://127.0.0.1:{port}/metrics", timeout=5.0)
    if code != 200:
        return None
    out = {"cpu": {}, "ctr": {}, "age": {}, "backend": {}, "gpus": set(), "rss": {}, "hbm": {}}
    for s in parse_text(body):
        d = s.label_dict()
        if s.name == "rocmdash_node_cpu_seconds_total":
            out["cpu"][d["process"]] = s.value
        elif s.name == "rocmdash_sampler_samples_total" and d.get("source") == "counter":
            out["ctr"][d["gpu_id"]] = s.value
            out["backend"][d["gpu_id"]] = d.get("backend")
        elif s.name == "rocmdash_sample_age_seconds" and d.get("source") == "counter":
            out["age"][d["gpu_id"]] = s.value
        elif s.name == "amd_gpu_gfx_activity":
            out["gpus"].add(d["gpu_id"])
        elif s.name == "rocmdash_self_rss_bytes":
            out["rss"][d["gpu_id"]] = s.value
        elif s.name == "rocmdash_self_hbm_bytes":
            out["hbm"][d["gpu_id"]] = s.value
    return out


def main() -> int:
    from _supervisor_helpers import free_port, start_node, stop_node

    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, default=8)
    ap.add_argument("--counter-daemon", default="on", choices=["on", "off", "auto"])
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--counters", default="auto")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    port = free_port()
    log = os.path.join(ROOT, "gpurun_out", f"node_cpu_{args.nproc}_{args.counter_daemon}.log")
    os.makedirs(os.path.dirname(log), exist_ok=True)
    p = start_node(args.nproc, port, cpu=False, counter_daemon=args.counter_daemon, log_path=log,
                   serve_args=("--refresh-hz", "1", "--collective-timeout", "30", "--counters", args.counters),
                   env={"ROCMDASH_SMI_HZ": "10", "ROCMDASH_COUNTER_HZ": "100"})
    res = {"nproc": args.nproc, "counter_daemon": args.counter_daemon, "error": None}
    try:
        t_end = time.monotonic() + 240
        a = None
        while time.monotonic() < t_end:
            a = read(port)
            if a and len(a["gpus"]) == args.nproc and len(a["ctr"]) == args.nproc and min(a["ctr"].values()) > 200:
                break
            time.sleep(1.0)
        else:
            res["error"] = f"not every GPU up with counters: {a}"
            raise SystemExit
        time.sleep(2.0)
        a = read(port)
        ta = time.monotonic()
        print(f"[node_cpu_probe] measuring {args.seconds} s", flush=True)
        time.sleep(args.seconds)
        b = read(port)
        tb = time.monotonic()
        dt = tb - ta
        rate = {k: round((b["cpu"][k] - a["cpu"].get(k, 0.0)) / dt, 4) for k in b["cpu"]}
        res.update({
            "seconds": round(dt, 2),
            "node_cpu_seconds_per_s": rate,
            "node_cpu_seconds_per_s_total": round(sum(rate.values()), 4),
            "counter_rows_per_s_by_gpu": {g: round((b["ctr"][g] - a["ctr"][g]) / dt, 1) for g in sorted(b["ctr"])},
            "counter_age_s_by_gpu": b["age"],
            "counter_backend": sorted(set(b["backend"].values())),
            "rank_rss_mib": {g: round(v / 2**20, 1) for g, v in b["rss"].items()},
            "rank_hbm_mib": {g: round(v / 2**20, 1) for g, v in b["hbm"].items()},
        })
    except SystemExit:
        pass
    finally:
        rc = stop_node(p)
        res["rc"] = rc
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    return 0 if res["error"] is None else 1


if __name__ == "__main__":
    raise SystemExit(main())
