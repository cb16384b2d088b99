"""GPU-box probe: units of the SMU table's instantaneous PCIe bandwidth figure. Streams
pinned host -> device copies of known size for ~1 s while the SMI source samples, and
prints the column next to the measured copy rate."""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch

    from rocmdash.runtime import native

    nat = native.load()
    src = nat.make_smi_source(0, 0)
    ix = list(nat.SMI_FIELDS).index("amd_gpu_pcie_bandwidth")
    idle = [src.sample()[ix] for _ in range(50)]
    h = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    d = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    stop = threading.Event()
    vals = []

    def sampler():
        while not stop.is_set():
            vals.append(float(src.sample()[ix]))
            time.sleep(0.002)

    th = threading.Thread(target=sampler)
    th.start()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 1.5:
        d.copy_(h, non_blocking=True)
        n += 1
        if n % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stop.set()
    th.join()
    v = np.array(vals)
    print(json.dumps({"h2d_GBps": round(n * (1 << 30) / dt / 1e9, 2), "idle_p50": float(np.median(idle)),
                      "during_p50": float(np.median(v)), "during_p90": float(np.percentile(v, 90)),
                      "during_max": float(v.max()), "samples": len(v)}))


if __name__ == "__main__":
    main()
