"""GPU-box probe: do the SMU-table read and the device-counter read slow each other
down? In one process with our runtime (counters registered before HIP init, as in the
bench) time each source's read alone, then both concurrently (agent.sample(): the
counter read on its worker thread, the table read on this one), then both in
sequence. Run as several fresh processes: the bench's fast / slow states
 should show up here if they are contention between the two reads."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def p50(xs):
    xs = sorted(xs)
    return round(xs[len(xs) // 2] * 1e6, 1)


def main():
    from rocmdash.runtime import native

    native.load()
    native.enable_counters()
    import torch

    from rocmdash.runtime.agent import GpuAgent

    torch.zeros(1, device="cuda")
    agent = GpuAgent(0, source="hw", counters="hw")
    smi, ctr = agent.samplers[0], agent.samplers[1]
    n = 1500
    res = {"env": {k: os.environ[k] for k in ("HSA_ENABLE_INTERRUPT",) if k in os.environ}}
    quick = os.environ.get("PROBE_QUICK") == "1"
    for name, fn in ((("ctr_alone", lambda: ctr.sample_once()),) if quick else (
        ("smi_alone", lambda: smi.sample_once()),
        ("ctr_alone", lambda: ctr.sample_once()),
        ("both_concurrent", agent.sample),
        ("both_serial", lambda: (ctr.sample_once(), smi.sample_once())),
        ("smi_alone_again", lambda: smi.sample_once()),
        ("ctr_alone_again", lambda: ctr.sample_once()),
    )):
        for _ in range(50):
            fn()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        res[name] = p50(ts)
    # concurrent again, but the table read starts only once the counter read is done
    # on its worker thread's side of the hand-off: staggered by a fixed delay
    for delay_us in (() if quick else (20, 40, 60)):
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            ctr.request()
            t_wait = t0 + delay_us * 1e-6
            while time.perf_counter() < t_wait:
                pass
            smi.sample_once()
            ctr.wait()
            ts.append(time.perf_counter() - t0)
        res[f"staggered_{delay_us}us"] = p50(ts)
    st = agent.sampler_stats()
    res["sampler_mean_us"] = [round(s["mean_us"], 1) for s in st]
    print(json.dumps(res), flush=True)
    agent.close()


if __name__ == "__main__":
    main()
