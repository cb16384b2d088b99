"""Does any HSA runtime knob shrink a process's ~347 MiB of driver-side device memory
(its GPU context and one hardware queue, profiles/r06/footprint/)? Round 5 tried the
scratch, fragment-allocator, AQL-queue-size and staging knobs (profiles/r05/footprint/);
this tries the rest of libhsa-runtime64's list that could touch per-process or per-queue
state. Each variant: a fresh process brings torch up and launches one kernel under
GPU_MAX_HW_QUEUES=1 + HSA_SCRATCH_SINGLE_LIMIT=1 MiB (the supervisor's environment) plus
the variant; the device's used VRAM is read before and while it holds its memory.

    python tools/probes/probe_hsa_env.py OUT.jsonl
"""

import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CHILD = r"""
import sys, time, torch
x = torch.ones(1 << 20, device='cuda'); (x * 2).sum().item()
print('ready', flush=True)
time.sleep(4.0)
"""

VARIANTS = [
    {},
    {"HSA_DISABLE_PC_SAMPLING": "1"},
    {"HSA_ALLOCATE_QUEUE_DEV_MEM": "0"},
    {"HSA_ALLOCATE_QUEUE_DEV_MEM": "1"},
    {"HSA_ENABLE_SCRATCH_ALT": "0"},
    {"HSA_MAX_QUEUES": "1"},
    {"HSA_DISABLE_COREDUMP_ON_EXCEPTION": "1"},
    {"HSA_CU_MASK_SKIP_INIT": "1"},
    {"HSA_ENABLE_DEBUG": "0"},
    {"HSA_DISABLE_CACHE": "1"},
]


def main():
    from rocmdash.runtime.footprint import drm_vram_by_bdf, sysfs_vram_used
    from rocmdash.runtime.topology import bdf_of_hip_device

    out_path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/hsa_env.jsonl"
    bdf = bdf_of_hip_device(0)
    lines = []
    for v in VARIANTS:
        env = dict(os.environ, PYTHONPATH=ROOT, GPU_MAX_HW_QUEUES="1", HSA_SCRATCH_SINGLE_LIMIT="1048576", **v)
        time.sleep(1.0)
        u0 = sysfs_vram_used(bdf)
        p = subprocess.Popen([sys.executable, "-c", CHILD], env=env, stdout=subprocess.PIPE, text=True)
        ok = p.stdout.readline().strip() == "ready"
        time.sleep(0.5)
        u1 = sysfs_vram_used(bdf)
        own = sum(drm_vram_by_bdf(p.pid).values())
        p.wait(timeout=60)
        rec = {"env": v, "ok": ok, "device_growth_mib": round((u1 - u0) / 2**20, 1),
               "own_buffers_mib": round(own / 2**20, 1), "driver_side_mib": round((u1 - u0 - own) / 2**20, 1)}
        print(json.dumps(rec), flush=True)
        lines.append(rec)
    with open(out_path, "w") as f:
        for r in lines:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
