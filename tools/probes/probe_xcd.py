"""GPU-box probe: per-XCD fields of the SMU metrics table (v1.8). Prints the raw table's
candidate per-XCD words (gfx clocks u16[8] @296, busy u32[8] @340, busy accumulators
u64[8] @464) next to amd-smi's decoding (current_gfxclks, xcp_stats.gfx_busy_inst /
gfx_busy_acc), idle and under a bf16 GEMM load, so the offsets can be pinned."""
import json
import os
import struct
import sys
import threading
import time

sys.path.insert(0, "/opt/rocm/share/amd_smi")


def main():
    import amdsmi
    import torch

    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
    bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)
    path = f"/sys/bus/pci/devices/{bdf}/gpu_metrics"

    def raw():
        with open(path, "rb") as f:
            b = f.read()
        return {"clk296": list(struct.unpack_from("<8H", b, 296)),
                "busy340": list(struct.unpack_from("<8I", b, 340)),
                "acc464": list(struct.unpack_from("<8Q", b, 464)),
                "ts288": struct.unpack_from("<Q", b, 288)[0]}

    def smi():
        m = amdsmi.amdsmi_get_gpu_metrics_info(h)
        keep = {}
        for k in ("current_gfxclks", "xcp_stats.gfx_busy_inst", "xcp_stats.gfx_busy_acc", "average_gfx_activity",
                  "num_partition"):
            keep[k] = m.get(k)
        return keep

    def both(tag):
        r1 = raw()
        s = smi()
        r2 = raw()
        print(json.dumps({"tag": tag, "raw_before": r1, "smi": s, "raw_after": r2}, default=str), flush=True)

    for i in range(3):
        both(f"idle{i}")
        time.sleep(0.05)
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    stop = threading.Event()

    def load():
        while not stop.is_set():
            for _ in range(20):
                a @ b
            torch.cuda.synchronize()

    th = threading.Thread(target=load)
    th.start()
    time.sleep(0.5)
    for i in range(4):
        both(f"gemm{i}")
        time.sleep(0.1)
    stop.set()
    th.join()
    # an 8-workgroup kernel: one XCD's worth of work at most (workgroups go round-robin
    # over the XCDs, so this lights a few XCDs, not all)
    x = torch.empty(8 * 256, device="cuda")
    stop.clear()

    def small():
        while not stop.is_set():
            for _ in range(200):
                x.add_(1.0)
            torch.cuda.synchronize()

    th = threading.Thread(target=small)
    th.start()
    time.sleep(0.3)
    for i in range(2):
        both(f"small{i}")
        time.sleep(0.1)
    stop.set()
    th.join()
    amdsmi.amdsmi_shut_down()


if __name__ == "__main__":
    main()
