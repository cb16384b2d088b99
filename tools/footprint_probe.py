#!/usr/bin/env python3
"""The node service's own cost on the GPU node it watches (VERDICT r02 "missing" 3).

Starts ``rocmdash.serve`` at the production rates (amd-smi 10 Hz, device counters
100 Hz, one node refresh per second, the DaemonSet's flags), waits for it to serve, and
reads its own footprint series twice, ``--seconds`` apart, from ``/metrics``:

  rocmdash_self_hbm_bytes{gpu_id}          process HBM (KFD per-process accounting)
  rocmdash_self_rss_bytes{gpu_id}          resident host memory
  rocmdash_self_cpu_seconds_total{gpu_id}  CPU seconds of all threads -> CPU per wall second
  rocmdash_self_hbm_stage_bytes{stage}     rank 0's HBM after each start-up stage

    python tools/footprint_probe.py [--world 2] [--seconds 10] [--out file.json]

``--world N`` > GPUs oversubscribes (ROCMDASH_OVERSUBSCRIBE: N rank processes on the
GPU, RCCL over sockets) - the per-rank cost of the N-rank service incl. its communicator.
Prints one JSON line."""

from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scrape(url):
    from rocmdash.prom.exposition import parse_text

    with urllib.request.urlopen(url, timeout=5) as r:
        body = r.read().decode()
    out = {}
    for smp in parse_text(body):
        if smp.name.startswith("rocmdash_self_") or smp.name in ("rocmdash_gather_native", "rocmdash_node_ranks"):
            d = smp.label_dict()
            out[(smp.name, d.get("gpu_id"), d.get("stage") or d.get("class"))] = smp.value
    return out


def _proc_tree(pid: int) -> list:
    """pid and all its descendants (torchrun -> rank processes)."""
    out, todo = [], [pid]
    while todo:
        p = todo.pop()
        out.append(p)
        try:
            for t in os.listdir(f"/proc/{p}/task"):
                with open(f"/proc/{p}/task/{t}/children") as f:
                    todo += [int(c) for c in f.read().split()]
        except OSError:
            pass
    return out


def _thread_cpu(pids) -> dict:
    """{(pid, thread name): CPU seconds} of every thread of these processes."""
    tck = os.sysconf("SC_CLK_TCK")
    out = {}
    for p in pids:
        try:
            tids = os.listdir(f"/proc/{p}/task")
        except OSError:
            continue
        for t in tids:
            try:
                with open(f"/proc/{p}/task/{t}/stat") as f:
                    st = f.read()
            except OSError:
                continue
            name = st[st.index("(") + 1:st.rindex(")")]
            fields = st[st.rindex(")") + 2:].split()
            # one entry per thread: (pid, tid, name); tid order is creation order
            key = (p, int(t), name + (" [main]" if int(t) == p else ""))
            out[key] = (int(fields[11]) + int(fields[12])) / tck
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--source", default="auto")
    ap.add_argument("--counters", default="auto")
    ap.add_argument("--node-window", type=int, default=1)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)

    port = _free_port()
    serve = ["-m", "rocmdash.serve", "--host", "127.0.0.1", "--port", str(port), "--refresh-hz", "1",
             "--source", args.source, "--counters", args.counters]
    if args.node_window:
        serve.append("--node-window")
    env = dict(os.environ, PYTHONPATH=ROOT, ROCMDASH_SMI_HZ="10", ROCMDASH_COUNTER_HZ="100")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    if args.world > 1:
        import torch

        if torch.cuda.device_count() < args.world:
            env["ROCMDASH_OVERSUBSCRIBE"] = "1"
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.world),
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *serve]
    else:
        cmd = [sys.executable, *serve]
    log_path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"footprint_serve_{port}.log")
    log = open(log_path, "w")
    t_start = time.monotonic()
    proc = subprocess.Popen(cmd, cwd=ROOT, stdout=log, stderr=subprocess.STDOUT, env=env, start_new_session=True)
    url = f"http://127.0.0.1:{port}/metrics"
    res = {}
    try:
        deadline = time.monotonic() + 240
        first = None
        while time.monotonic() < deadline:
            if proc.poll() is not None:
                raise RuntimeError(f"service exited with {proc.returncode}")
            try:
                m = _scrape(url)
                if sum(1 for k in m if k[0] == "rocmdash_self_cpu_seconds_total" and k[2] == "normal") >= args.world:
                    first = m
                    break
            except OSError:
                pass
            time.sleep(0.5)
        if first is None:
            raise RuntimeError("no footprint series within 240 s")
        t_ready = time.monotonic() - t_start
        time.sleep(2.0)  # past the start-up refreshes
        pids = _proc_tree(proc.pid)
        a, ta = _scrape(url), time.monotonic()
        th_a = _thread_cpu(pids)
        time.sleep(args.seconds)
        b, tb = _scrape(url), time.monotonic()
        th_b = _thread_cpu(pids)
        busy = sorted(((th_b[k] - th_a.get(k, 0.0)) / (tb - ta), k) for k in th_b)[::-1]
        order = sorted(th_b)  # by (pid, tid): creation order within a process
        threads = [{"pid": k[0], "tid": k[1], "thread": k[2], "created_nth": order.index(k),
                    "cpu_per_wall_s": round(v, 4)} for v, k in busy[:8] if v > 0.001]
        named = [{"tid": k[1], "thread": k[2], "created_nth": order.index(k)} for k in order
                 if k[2].startswith("rd-") or "[main]" in k[2]]
        gpus = sorted({k[1] for k in b if k[0] == "rocmdash_self_cpu_seconds_total"})
        per = {}
        def rate(g, cls):
            k = ("rocmdash_self_cpu_seconds_total", g, cls)
            return round((b[k] - a[k]) / (tb - ta), 4) if k in a and k in b else None

        for g in gpus:
            per[g] = {
                "hbm_mib": round(b.get(("rocmdash_self_hbm_bytes", g, None), float("nan")) / 2**20, 1),
                "rss_mib": round(b.get(("rocmdash_self_rss_bytes", g, None), float("nan")) / 2**20, 1),
                "cpu_per_wall_s": rate(g, "normal"),  # normal scheduling class: taken from workloads
                "idle_class_cpu_per_wall_s": rate(g, "idle"),  # SCHED_IDLE: idle CPUs only
                "native_gather": b.get(("rocmdash_gather_native", g, None)),
            }
        stages = {k[2]: round(v / 2**20, 1) for k, v in b.items() if k[0] == "rocmdash_self_hbm_stage_bytes"}
        res = {"world": args.world, "oversubscribed": env.get("ROCMDASH_OVERSUBSCRIBE") == "1",
               "rates": "amd-smi 10 Hz, counters 100 Hz, node refresh 1 Hz" + (", node window" if args.node_window else ""),
               "seconds": round(tb - ta, 2), "time_to_first_metrics_s": round(t_ready, 2), "per_gpu": per,
               "rank0_hbm_mib_after_stage": stages,
               "max_hbm_mib": max(p["hbm_mib"] for p in per.values()),
               "max_rss_mib": max(p["rss_mib"] for p in per.values()),
               "max_cpu_per_wall_s": max(p["cpu_per_wall_s"] for p in per.values() if p["cpu_per_wall_s"] is not None),
               "busiest_threads": threads, "threads_total": len(order), "landmark_threads": named,
               "kfd_per_process": os.path.isdir(f"/sys/class/kfd/kfd/proc/{pids[-1]}")}
    finally:
        if proc.poll() is None:
            os.killpg(proc.pid, signal.SIGTERM)
            try:
                proc.wait(timeout=60)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
                proc.wait()
        log.close()
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
