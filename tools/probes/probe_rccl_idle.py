"""Does an idle RCCL communicator slow this process's GPU round trips?

Measures, before and after a one-rank NCCL (RCCL) process group is created (eager
init, no collective issued): p50 of a device-counter read (rocprofiler-sdk), of a
tiny kernel + stream synchronize, of a pinned-host-output kernel + synchronize; then
which threads of the process burn CPU while idle (/proc/self/task). Env vars under
test are passed through by the caller."""

import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def threads():
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                parts = f.read().rsplit(")", 1)
            name = parts[0].split("(", 1)[1]
            fields = parts[1].split()
            out[tid] = (name, int(fields[11]) + int(fields[12]))  # utime + stime (ticks)
        except OSError:
            pass
    return out


def native_choice():
    from rocmdash.runtime.placement import choice

    c = choice()
    return None if c is None else c.get("node")


def main():
    cpus = sorted(os.sched_getaffinity(0))
    print(json.dumps({"phase": "start", "affinity": len(cpus), "first": cpus[0], "last": cpus[-1]}), flush=True)
    from rocmdash.runtime import native

    nat = native.load()
    native.enable_counters()
    cpus = sorted(os.sched_getaffinity(0))
    print(json.dumps({"phase": "pinned", "affinity": len(cpus), "first": cpus[0], "last": cpus[-1]}), flush=True)
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    early = os.environ.get("PROBE_ORDER", "late") == "early"
    if early:  # bench.py's order: the group comes up before anything else touches the GPU
        kw = {"backend": "nccl", "rank": 0, "world_size": 1, "store": dist.HashStore(), "device_id": dev}
        dist.init_process_group(**kw)
        cpus = sorted(os.sched_getaffinity(0))
        print(json.dumps({"phase": "group_created_early", "affinity": len(cpus), "first": cpus[0], "last": cpus[-1],
                          "pinned_by_placement": native_choice()}), flush=True)
    bdf = int(nat.hip_device_bdf(0))
    src = nat.make_counter_source(bdf, 0) if native.counters_ready() else None
    x = torch.zeros(16, device=dev)
    host = torch.zeros(16, pin_memory=True)

    def measure(tag):
        res = {}
        if src is not None:
            for _ in range(50):
                src.sample()
            ts = []
            for _ in range(500):
                t0 = time.perf_counter()
                src.sample()
                ts.append(time.perf_counter() - t0)
            res["counter_read_us"] = round(statistics.median(ts) * 1e6, 1)
        s = torch.cuda.current_stream()
        ts = []
        for _ in range(500):
            t0 = time.perf_counter()
            x.add_(1.0)
            s.synchronize()
            ts.append(time.perf_counter() - t0)
        res["kernel_sync_us"] = round(statistics.median(ts) * 1e6, 1)
        ts = []
        for _ in range(500):
            t0 = time.perf_counter()
            host.copy_(x, non_blocking=True)
            s.synchronize()
            ts.append(time.perf_counter() - t0)
        res["d2h_sync_us"] = round(statistics.median(ts) * 1e6, 1)
        print(json.dumps({"phase": tag, **res}), flush=True)

    measure("before")
    if early:
        time.sleep(2.0)
        th = threads()
        print(json.dumps({"phase": "threads", "n": len(th)}))
        dist.destroy_process_group()
        time.sleep(0.5)
        measure("after_destroy")
        return
    kw = {"backend": "nccl", "rank": 0, "world_size": 1, "store": dist.HashStore()}
    if os.environ.get("PROBE_EAGER", "1") == "1":
        kw["device_id"] = dev
    dist.init_process_group(**kw)
    if os.environ.get("PROBE_COLLECTIVE", "0") == "1":
        out = torch.empty(1, 16, device=dev)
        dist.all_gather_into_tensor(out, x)
        torch.cuda.synchronize()
    time.sleep(0.5)
    th0 = threads()
    time.sleep(2.0)
    th1 = threads()
    busy = sorted(((th1[t][1] - th0.get(t, ("", th1[t][1]))[1], th1[t][0]) for t in th1), reverse=True)[:6]
    print(json.dumps({"phase": "idle_threads_ticks_2s", "busy": busy, "n_threads": len(th1)}), flush=True)
    measure("after_group")
    dist.destroy_process_group()
    time.sleep(0.5)
    measure("after_destroy")


if __name__ == "__main__":
    main()
