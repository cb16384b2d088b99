"""Node-total CPU and memory of the supervised service at production rates (VERDICT r04
items 3 and 6): ``rocmdash.runtime.nodemeasure.measure_production`` from the command
line. One JSON line.

    ROCMDASH_OVERSUBSCRIBE=1 python tools/node_cpu_probe.py --nproc 8 --counter-daemon on
"""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    from rocmdash.runtime.nodemeasure import measure_production

    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, default=8)
    ap.add_argument("--counter-daemon", default="on", choices=["on", "off", "auto"])
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--counters", default="auto")
    ap.add_argument("--cpu", action="store_true", help="CPU ranks with synthetic sources (a rehearsal)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    log = os.path.join(ROOT, "gpurun_out", f"node_cpu_{args.nproc}_{args.counter_daemon}.log")
    os.makedirs(os.path.dirname(log), exist_ok=True)
    extra = ("--source", "synthetic") if args.cpu else ()
    res = measure_production(args.nproc, seconds=args.seconds, counter_daemon=args.counter_daemon,
                             counters="synthetic" if args.cpu else args.counters, log_path=log, cpu=args.cpu,
                             extra_serve_args=extra)
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    return 0 if res["error"] is None else 1


if __name__ == "__main__":
    raise SystemExit(main())
