"""Read cost AND byte accuracy of one device-counter set, in one process.

    python tools/probes/probe_counter_accuracy.py SET [--n 1000]

SET is a comma-separated counter list. Prints one JSON line: the read's p10/p50/p90
over n back-to-back reads, the configured counters / instance records, and the HBM
read / write series against kernels of known traffic (csrc/calib.hip): random 32 B
reads (one 128 B line each), 64 B and 32 B stores 256 B apart, a 64 MiB (MALL) and a
1 GiB copy. Counters are configured before HIP starts, so each set needs its own
process (tools/probes/run_counter_ab.sh alternates them)."""

import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    names = sys.argv[1].split(",")
    n = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[2] == "--n" else 1000
    from rocmdash.runtime import native

    nat = native.load()
    ok, st = native.enable_counters(names, only_device=0)
    import torch

    bdf = int(nat.hip_device_bdf(0))
    src = nat.make_counter_source(bdf, 0)
    src.sample()
    lat = []
    for _ in range(n):
        t0 = time.perf_counter()
        src.sample()
        lat.append((time.perf_counter() - t0) * 1e6)
    lat.sort()
    out = {"counters": names, "ok": ok, "status": st, "set": src.counts(),
           "p50_us": round(statistics.median(lat), 1), "p10_us": round(lat[len(lat) // 10], 1),
           "p90_us": round(lat[9 * len(lat) // 10], 1)}
    stream = torch.cuda.current_stream().cuda_stream
    big = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")
    big.zero_()
    sink = torch.empty(1 << 18, dtype=torch.float32, device="cuda")

    def measure(fn, rd_call, wr_call, secs=0.3):
        fn(0)
        torch.cuda.synchronize()
        src.sample()
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < secs:
            for _ in range(10):
                fn(k)
                k += 1
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        r = src.sample().tolist()
        true_rd, true_wr = k * rd_call / dt / 1e9, k * wr_call / dt / 1e9
        return {"rd": round(r[1], 2), "wr": round(r[2], 2), "true_rd": round(true_rd, 2), "true_wr": round(true_wr, 2),
                "rd_ratio": round(r[1] / true_rd, 3) if true_rd else None,
                "wr_ratio": round(r[2] / true_wr, 3) if true_wr else None}

    G = 1 << 24
    out["gather32"] = measure(lambda i: nat.calib_gather32(big.data_ptr(), big.numel(), sink.data_ptr(),
                                                           sink.numel() * 4, G, 7 + i, stream), 128 * G, 4 * (G // 256))
    S = 1 << 22
    out["store64"] = measure(lambda i: nat.calib_store64(big.data_ptr(), big.numel(), S, stream), 0, 64 * S)
    out["store32"] = measure(lambda i: nat.calib_store32(big.data_ptr(), big.numel(), S, stream), 0, 32 * S)
    m = 64 << 20
    x, y = big[:m], big[m:2 * m]
    out["copy_mall"] = measure(lambda i: y.copy_(x), m, m)
    g = 1 << 30
    out["copy_1g"] = measure(lambda i: big[g:].copy_(big[:g]), g, g)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
