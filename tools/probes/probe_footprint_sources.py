import glob, os, json, subprocess, sys
sys.path.insert(0, os.getcwd())
from rocmdash.runtime.topology import bdf_of_hip_device
from rocmdash.runtime.agent import bdf_path
b = bdf_of_hip_device(0)
p = bdf_path(b) if b else None
out = {"bdf": hex(b) if b else None, "path": p, "exists": os.path.exists(p) if p else None}
try:
    out["vram_used_before"] = open(p + "/mem_info_vram_used").read().strip()
except Exception as e:
    out["vram_used_before"] = repr(e)
import torch
x = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
try:
    out["vram_used_after_256MiB"] = open(p + "/mem_info_vram_used").read().strip()
except Exception as e:
    out["vram_used_after_256MiB"] = repr(e)
free, total = torch.cuda.mem_get_info()
out["hip_used"] = total - free
out["kfd_files"] = {f: open(f).read().strip() for f in glob.glob(f"/sys/class/kfd/kfd/proc/{os.getpid()}/*") if "vram" in f}
out["drm_cards"] = sorted(glob.glob("/sys/class/drm/card*/device/mem_info_vram_used"))
print(json.dumps(out))
