"""Probe: which start-up step leaves a thread spinning a full core (footprint_probe.py
found one thread, created before the sampler threads, at ~1.0 CPU-second per second
whenever the device counters are live, at any counter rate)?

Stages, each followed by a 1.5 s window of per-thread CPU accounting:
  hip       native.load + enable_counters (tool registered) + HIP initialised
  source    make_counter_source(bdf, 0) (counting context configured and started)
  sampled   after 100 synchronous counter reads
  smi       after an amd-smi source is made too
Prints one JSON line: per stage, the threads that appeared and the busy ones.
"""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
TCK = os.sysconf("SC_CLK_TCK")


def threads():
    out = {}
    for t in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{t}/stat") as f:
                st = f.read()
        except OSError:
            continue
        name = st[st.index("(") + 1:st.rindex(")")]
        fields = st[st.rindex(")") + 2:].split()
        out[int(t)] = (name, (int(fields[11]) + int(fields[12])) / TCK, fields[0])
    return out


def window(label, seen, res, secs=1.5):
    a = threads()
    time.sleep(secs)
    b = threads()
    new = sorted(t for t in b if t not in seen)
    busy = sorted(((b[t][1] - a.get(t, (None, 0.0))[1]) / secs, t) for t in b)[::-1]
    res[label] = {
        "new_threads": [{"tid": t, "name": b[t][0]} for t in new],
        "busy": [{"tid": t, "name": b[t][0], "state": b[t][2], "cpu_per_s": round(v, 3)} for v, t in busy[:4] if v > 0.02],
        "threads": len(b),
    }
    seen.update(b)


def main():
    res = {}
    seen = set(threads())
    from rocmdash.runtime import native

    nat = native.load()
    ok, status = native.enable_counters(only_device=0)
    import torch

    torch.cuda.init()
    torch.empty(1, device="cuda")
    res["counters"] = [ok, status]
    window("hip", seen, res)
    bdf = int(nat.hip_device_bdf(0))
    src = nat.make_counter_source(bdf, 0)
    window("source", seen, res)
    for _ in range(100):
        src.sample()
    window("sampled", seen, res)
    smi = nat.make_smi_source(bdf, 0)
    smi.sample() if hasattr(smi, "sample") else None
    window("smi", seen, res)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
