"""Cost of one rocprofiler-sdk device-counting read as a function of the counter set.

    python tools/probes/probe_counter_cost.py GRBM_GUI_ACTIVE,TCC_EA0_RDREQ_sum [--n 300]

Counters are configured before HIP starts, so each set needs its own process
(tools/gpu_round.sh counterset runs several)."""

import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    names = sys.argv[1].split(",")
    n = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[2] == "--n" else 300
    from rocmdash.runtime import native

    nat = native.load()
    ok, st = native.enable_counters(names, only_device=0)
    import torch  # noqa: F401  (HIP init after the tool registered)

    bdf = int(nat.hip_device_bdf(0))
    src = nat.make_counter_source(bdf, 0)
    src.sample()
    lat = []
    for _ in range(n):
        t0 = time.perf_counter()
        src.sample()
        lat.append((time.perf_counter() - t0) * 1e6)
    lat.sort()
    print(json.dumps({"counters": names, "ok": ok, "status": st, "p50_us": round(statistics.median(lat), 1),
                      "p10_us": round(lat[len(lat) // 10], 1), "p90_us": round(lat[9 * len(lat) // 10], 1)}))


if __name__ == "__main__":
    main()
