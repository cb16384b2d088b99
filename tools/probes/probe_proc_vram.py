"""Per-process device memory without KFD's per-process sysfs (0 on the pool's boxes):
what each source says for a rank-like process and a counter-process-like one.

    python tools/probes/probe_proc_vram.py OUT.json

Starts, one after another, (a) a process that brings torch up and launches a kernel on a
second stream (a rank's HIP footprint), (b) the node counter process for device 0 with
synthetic-free hardware counters (rocprofiler-sdk queue), and reads for each pid, while it
holds its memory: DRM fdinfo (``/proc/<pid>/fdinfo/*``: ``drm-memory-vram``,
``drm-resident-*``, ``amd-*``), KFD's ``/sys/class/kfd/kfd/proc/<pid>/vram_*``, and the
device's ``mem_info_vram_used`` before / during / after. VERDICT r05 item 4."""

import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def fdinfo(pid: int) -> dict:
    out = {}
    for f in glob.glob(f"/proc/{pid}/fdinfo/*"):
        try:
            with open(f) as fh:
                txt = fh.read()
        except OSError:
            continue
        if "drm-driver" not in txt:
            continue
        client = None
        vals = {}
        for line in txt.splitlines():
            k, _, v = line.partition(":")
            v = v.strip()
            if k == "drm-client-id":
                client = v
            elif k.startswith(("drm-memory", "drm-resident", "drm-total", "drm-shared", "amd-", "drm-purgeable",
                               "drm-active")):
                vals[k] = v
        out[f"{os.path.basename(f)}:{client}"] = vals
    return out


def kfd(pid: int) -> dict:
    out = {}
    for f in glob.glob(f"/sys/class/kfd/kfd/proc/{pid}/*"):
        if os.path.isdir(f):
            continue
        try:
            with open(f) as fh:
                out[os.path.basename(f)] = fh.read().strip()[:200]
        except OSError as e:
            out[os.path.basename(f)] = f"error: {e}"
    return out


def used(bdf):
    from rocmdash.runtime.footprint import sysfs_vram_used

    return sysfs_vram_used(bdf)


RANK = r"""
import sys, time, torch
x = torch.ones(1 << 20, device='cuda'); s = torch.cuda.Stream()
with torch.cuda.stream(s):
    y = x * 2
torch.cuda.synchronize()
print('ready', flush=True)
time.sleep(float(sys.argv[1]))
"""


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/proc_vram.json"
    from rocmdash.runtime.topology import bdf_of_hip_device

    bdf = bdf_of_hip_device(0)
    res = {"bdf": bdf, "runs": []}
    env = dict(os.environ, PYTHONPATH=ROOT)
    for kind in ("rank", "rank_lean", "counterd", "counterd_lean"):
        e = dict(env)
        if kind.endswith("lean"):
            e.update(GPU_MAX_HW_QUEUES="1", HSA_SCRATCH_SINGLE_LIMIT="1048576")
        u0 = used(bdf)
        if kind.startswith("rank"):
            p = subprocess.Popen([sys.executable, "-c", RANK, "8"], env=e, stdout=subprocess.PIPE, text=True)
            p.stdout.readline()
            time.sleep(1.0)
        else:
            d = f"/tmp/rocmdash-probe-ctr-{os.getpid()}"
            os.makedirs(d, exist_ok=True)
            p = subprocess.Popen([sys.executable, "-m", "rocmdash.runtime.counterd", "--dir", d, "--devices", "0",
                                  "--hz", "100"], env=e, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            t0 = time.monotonic()
            while time.monotonic() - t0 < 60 and not os.path.exists(os.path.join(d, "status.json")):
                time.sleep(0.2)
            time.sleep(1.5)
        u1 = used(bdf)
        rec = {"kind": kind, "pid": p.pid, "device_used_growth_mib": round((u1 - u0) / 2**20, 1) if u0 and u1 else None,
               "fdinfo": fdinfo(p.pid), "kfd": kfd(p.pid)}
        p.terminate()
        try:
            p.wait(timeout=20)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
        time.sleep(1.0)
        u2 = used(bdf)
        rec["device_used_released_mib"] = round((u1 - u2) / 2**20, 1) if u1 and u2 else None
        res["runs"].append(rec)
        print(json.dumps({k: rec[k] for k in ("kind", "device_used_growth_mib", "device_used_released_mib")}),
              flush=True)
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
