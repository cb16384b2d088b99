"""Where a rank's device memory goes at world 1 / 2 / 8 (the 8-rank
rehearsal's 2.4-4.2 GiB per rank).

    ROCMDASH_OVERSUBSCRIBE=1 python -m torch.distributed.run --nproc-per-node 8 \\
        --master-addr 127.0.0.1 --master-port 29571 tools/probes/probe_rank_vram_world.py

Every rank goes through the same start-up stages together (gloo barriers): HIP up with
its first kernel, the GPU agent (synthetic sources, one refresh), the native RCCL
communicator, one all-gather through it. After each stage rank 0 reads the device's used
VRAM (sysfs) and every rank its own buffers (DRM fdinfo, rocmdash.runtime.footprint).
Rank 0 prints one JSON line per stage: the device growth since the start, the ranks'
own buffers summed, and what no process's buffers explain (driver-side state), per
rank. Run it under the supervisor's environment (LEAN_RUNTIME_ENV) to see the service's
numbers."""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    from rocmdash.runtime import native

    native.load()
    import torch
    import torch.distributed as dist

    from rocmdash.parallel.node import NodeAggregator, dist_env_from_environ
    from rocmdash.runtime.footprint import drm_vram_by_bdf, sysfs_vram_used
    from rocmdash.runtime.topology import bdf_of_hip_device

    bdf = bdf_of_hip_device(0)
    base = sysfs_vram_used(bdf)  # before this rank's HIP start (the others may be starting too)
    env = dist_env_from_environ(prefer_gpu=True, timeout_s=300, world1_group=True)
    rank, world = env.rank, env.world_size
    gbase = [None]

    def stage(name):
        dist.barrier()
        time.sleep(0.5)
        used = sysfs_vram_used(bdf) if rank == 0 else None
        own = sum(drm_vram_by_bdf(os.getpid()).values())
        got = [None] * world
        dist.all_gather_object(got, {"rank": rank, "own": own, "used": used})
        if rank == 0:
            if gbase[0] is None:
                gbase[0] = min(base, used)
            growth = used - gbase[0]
            owns = [g["own"] for g in got]
            print(json.dumps({"stage": name, "world": world, "device_growth_mib": round(growth / 2**20, 1),
                              "own_buffers_mib_by_rank": [round(o / 2**20, 1) for o in owns],
                              "unattributed_mib_per_rank": round((growth - sum(owns)) / world / 2**20, 1),
                              "env": {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES", "NCCL_BUFFSIZE",
                                                                     "NCCL_MAX_NCHANNELS", "HSA_SCRATCH_SINGLE_LIMIT")}}),
                  flush=True)

    stage("gloo")
    x = torch.ones(1 << 20, device=env.device)
    (x * 2).sum().item()
    stage("hip_first_kernel")
    from rocmdash.runtime.agent import GpuAgent

    agent = GpuAgent(env.device.index, source="synthetic", counters="synthetic", use_gpu=True, seed=1000 + rank)
    agent.prefill(256)
    agent.refresh()
    torch.cuda.synchronize()
    stage("agent")
    agg = NodeAggregator(force_collective=world == 1)
    ok = agg.enable_native(env.device)
    stage("rccl_comm" + ("" if ok else "_failed"))
    if ok:
        blk = agent.export_window() if hasattr(agent, "export_window") else x[:1024]
        agg.all_gather(blk)
        torch.cuda.synchronize()
        stage("rccl_allgather")
        agg.native.close()
    agent.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
