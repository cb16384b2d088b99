"""Probe: is the NUMA "slow state" of the device-counter read (profiles/r01/numa_ab.txt:
~140 us vs ~75 us, fixed for a process's life by the node it started HSA on) the
placement of the runtime's busy-polling async-events thread (rocmdash/runtime/threads.py),
which inherits the CPU mask of the thread that started HSA?

Starts HSA unpinned, finds the spinner, then moves ONLY the spinner between NUMA nodes
(and onto single cores) in the same process and times 200 counter reads from the main
thread for each placement; then the same with the reading thread moved too.
Prints one JSON line.
"""

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def reads(src, n=200, warm=30):
    for _ in range(warm):
        src.sample()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        src.sample()
        ts.append((time.perf_counter() - t0) * 1e6)
    return round(statistics.median(ts), 1)


def main():
    os.environ["ROCMDASH_INIT_PLACEMENT"] = "0"
    from rocmdash.runtime import native
    from rocmdash.runtime.placement import numa_nodes
    from rocmdash.runtime.threads import busy_foreign_threads

    nat = native.load()
    ok, status = native.enable_counters(only_device=0)
    import torch

    torch.cuda.init()
    torch.empty(1, device="cuda")
    bdf = int(nat.hip_device_bdf(0))
    src = nat.make_counter_source(bdf, 0)
    nodes = numa_nodes()
    spin = busy_foreign_threads(0.3)
    res = {"counters": [ok, status], "nodes": {n: len(c) for n, c in nodes.items()},
           "spinners": [(t, n, round(r, 2)) for t, n, r in spin], "gpu_numa": None}
    try:
        with open(f"/sys/bus/pci/devices/{bdf >> 32:04x}:{(bdf >> 8) & 0xff:02x}:{(bdf >> 3) & 0x1f:02x}.{bdf & 7:x}/numa_node") as f:
            res["gpu_numa"] = int(f.read())
    except OSError:
        pass
    me = os.getpid()
    allcpus = sorted(os.sched_getaffinity(0))
    res["unpinned"] = reads(src)
    if not spin:
        print(json.dumps(res))
        return
    tid = spin[0][0]
    out = {}
    for n, cpus in nodes.items():
        os.sched_setaffinity(tid, cpus)
        out[f"spinner_node{n}"] = reads(src)
        os.sched_setaffinity(tid, [cpus[len(cpus) // 2]])
        out[f"spinner_core_node{n}"] = reads(src)
        for m, cpus2 in nodes.items():  # reader moved as well
            os.sched_setaffinity(me, cpus2)
            os.sched_setaffinity(tid, cpus)
            out[f"spinner_node{n}_reader_node{m}"] = reads(src)
        os.sched_setaffinity(me, allcpus)
    os.sched_setaffinity(tid, allcpus)
    out["back_unpinned"] = reads(src)
    res["p50_us"] = out
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
