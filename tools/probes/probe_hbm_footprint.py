"""What holds the exporter rank's HBM (487 MiB right after HIP /
torch start-up, 667 MiB in all). Each stage runs in a FRESH process; the device's used
VRAM (amdgpu sysfs, whole device - run alone on the box) is read before the process
starts anything and after each step inside it. One JSON line per stage.

    python tools/probes/probe_hbm_footprint.py [--hip-probe build/probe_hip_init]
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CHILD = r"""
import json, os, sys, time
sys.path.insert(0, ROOT)
from rocmdash.runtime.footprint import sysfs_vram_used
from rocmdash.runtime.topology import bdf_of_hip_device
bdf = bdf_of_hip_device(0)
# the previous process's memory is released asynchronously: wait for a steady reading
prev = None
for _ in range(100):
    cur = sysfs_vram_used(bdf)
    if cur == prev:
        break
    prev = cur
    time.sleep(0.3)
marks = {"start": sysfs_vram_used(bdf)}
def mark(k):
    time.sleep(0.05)
    marks[k] = sysfs_vram_used(bdf)
stage = STAGE
if stage in ("torch", "torch_alloc"):
    import torch
    torch.cuda.init(); mark("torch.cuda.init")
    x = torch.empty(1, device="cuda"); torch.cuda.synchronize(); mark("first tensor")
    if stage == "torch_alloc":
        y = torch.empty(1 << 20, device="cuda"); (y + 1).sum().item(); mark("first elementwise kernel")
elif stage == "steps":
    from rocmdash.runtime import native
    nat = native.load()
    import torch
    nat.hip_device_bdf(0); mark("hip_device_bdf")
    torch.cuda.set_device(0); mark("torch.cuda.set_device")
    x = torch.empty(1, device="cuda"); torch.cuda.synchronize(); mark("torch.empty (allocator)")
    nat.set_pinned_host_rings(True)
    ring = nat.SeriesRing(16, 16384); mark("pinned ring (hipHostMalloc)")
    dws = nat.DeviceWindowSet(4096, 0); mark("DeviceWindowSet")
    dws.add_ring(ring); mark("add_ring")
    out = torch.empty((16, 8), device="cuda")
    ring.push_many(__import__("numpy").ones((64, 16), "float32"), __import__("numpy").arange(64, dtype="uint64"))
    dws.refresh(out.data_ptr(), torch.cuda.current_stream().cuda_stream, 50.0, 90.0, 99.0, 0)
    torch.cuda.synchronize(); mark("first rocmdash kernel")
    s2 = torch.cuda.Stream(); mark("torch.cuda.Stream()")
    with torch.cuda.stream(s2):
        (x + 1).sum().item()
    mark("first torch kernel on it")
    y = torch.empty(1 << 20, device="cuda"); y.mul_(2.0); torch.cuda.synchronize(); mark("second torch kernel")
elif stage == "counterd":  # the node counter process (hw counters of GPU 0), no torch
    import subprocess, tempfile
    d = tempfile.mkdtemp()
    cp = subprocess.Popen([sys.executable, "-m", "rocmdash.runtime.counterd", "--dir", d, "--devices", "0",
                           "--source", "hw", "--hz", "100"], cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT))
    time.sleep(8.0); mark("counterd up 8 s")
    cp.terminate(); cp.wait(30)
elif stage == "agent_node":  # a rank reading the counter process's rings (counters="node")
    import subprocess, tempfile
    d = tempfile.mkdtemp()
    cp = subprocess.Popen([sys.executable, "-m", "rocmdash.runtime.counterd", "--dir", d, "--devices", "0",
                           "--source", "hw", "--hz", "100"], cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT))
    time.sleep(8.0); mark("counterd up 8 s")
    os.environ["ROCMDASH_COUNTER_SHM"] = d
    from rocmdash.runtime import native
    nat = native.load(); nat.hip_device_bdf(0); mark("hip via rocmdash (hip_device_bdf)")
    import torch
    from rocmdash.runtime.agent import GpuAgent
    a = GpuAgent(0, counters="node"); mark("GpuAgent(counters=node)")
    a.prefill(64); a.refresh(); torch.cuda.synchronize(); mark("first refresh")
    a.close()
    cp.terminate(); cp.wait(30)
elif stage in ("native", "agent", "agent_counters"):
    from rocmdash.runtime import native
    nat = native.load(); mark("native.load")
    if stage == "agent_counters":
        native.enable_counters(); mark("enable_counters")
    nat.hip_device_bdf(0); mark("hip via rocmdash (hip_device_bdf)")
    if stage != "native":
        import torch
        from rocmdash.config import SamplerConfig
        from rocmdash.runtime.agent import GpuAgent
        a = GpuAgent(0, counters="hw" if stage == "agent_counters" else "off"); mark("GpuAgent")
        a.prefill(64); a.refresh(); torch.cuda.synchronize(); mark("first refresh")
        a.close()
print(json.dumps({"stage": stage, "bdf": bdf, "marks": marks,
                  "mib": {k: round((v - marks["start"]) / 2**20, 1) for k, v in marks.items() if v is not None and marks["start"] is not None}}))
"""


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--hip-probe", default=None)
    ap.add_argument("--stages", default="steps,torch,torch_alloc,native,agent,agent_counters,counterd,agent_node")
    args = ap.parse_args()
    from rocmdash.runtime.agent import bdf_path
    from rocmdash.runtime.topology import bdf_of_hip_device

    bdf = bdf_of_hip_device(0)
    if args.hip_probe:
        import torch

        path = bdf_path(bdf) + "/mem_info_vram_used"
        torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")
        # /opt/rocm's HIP runtime (7.2) and torch's bundled one (the runtime every rank uses)
        for env_extra in ({}, {"HIP_ENABLE_DEFERRED_LOADING": "0"}, {"LD_LIBRARY_PATH": torch_lib}):
            res = subprocess.run([args.hip_probe, path], capture_output=True, text=True, timeout=120,
                                 env=dict(os.environ, **env_extra))
            d = json.loads(res.stdout.strip().splitlines()[-1]) if res.returncode == 0 else {"rc": res.returncode,
                                                                                             "err": res.stderr[-500:]}
            if "start" in d:
                d["mib"] = {k: round((v - d["start"]) / 2**20, 1) for k, v in d.items() if k != "start"}
            print(json.dumps({"stage": "hip_only_cpp", "env": env_extra, **d}), flush=True)
    for st in args.stages.split(","):
        for env_extra in ({}, {"HIP_ENABLE_DEFERRED_LOADING": "0"}) if st == "torch" else ({},):
            code = CHILD.replace("ROOT", repr(ROOT)).replace("STAGE", repr(st))
            res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                                 env=dict(os.environ, **env_extra))
            line = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
            if res.returncode != 0 or not line:
                print(json.dumps({"stage": st, "env": env_extra, "rc": res.returncode, "err": res.stderr[-800:]}),
                      flush=True)
                continue
            d = json.loads(line[-1])
            d["env"] = env_extra
            print(json.dumps(d), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
