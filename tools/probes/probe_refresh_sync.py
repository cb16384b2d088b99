"""GPU-box probe: where the ~30 us of a world-1 refresh's device part goes. Times
agent.refresh(out=pinned host buffer) (host-side launch) and the wait for it, with
the wait done three ways: hipStreamSynchronize, a spin on hipEventQuery, and a spin on
a word the kernel writes into the pinned output (the 'count' column of the last row).
Live sources, one new sample per refresh, as in the bench."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def pct(xs, q):
    xs = sorted(xs)
    return round(xs[int(q * (len(xs) - 1))] * 1e6, 1)


def main():
    from rocmdash.runtime import native

    native.load()
    native.enable_counters()
    import torch

    from rocmdash.runtime.agent import GpuAgent

    agent = GpuAgent(0)
    agent.prefill()
    host = torch.empty(agent.out.shape, dtype=torch.float32, pin_memory=True)
    stream = torch.cuda.current_stream()
    res = {}
    n = 1500
    for mode in ("stream_sync", "event_spin", "stream_sync", "event_spin"):
        launch, wait = [], []
        ev = torch.cuda.Event()
        for i in range(n + 50):
            agent.sample()
            t0 = time.perf_counter()
            agent.refresh(out=host)
            t1 = time.perf_counter()
            if mode == "stream_sync":
                stream.synchronize()
            else:
                ev.record(stream)
                while not ev.query():
                    pass
            t2 = time.perf_counter()
            if i >= 50:
                launch.append(t1 - t0)
                wait.append(t2 - t1)
        res.setdefault(mode, []).append({"launch_p50_us": pct(launch, 0.5), "wait_p50_us": pct(wait, 0.5),
                                         "wait_p90_us": pct(wait, 0.9)})
    st = agent.dws.stats() if hasattr(agent.dws, "stats") else {}
    res["dws"] = {k: st[k] for k in list(st)[:8]} if isinstance(st, dict) else None
    print(json.dumps(res), flush=True)
    agent.close()


if __name__ == "__main__":
    main()
