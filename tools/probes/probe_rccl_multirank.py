"""Probe: can N RCCL ranks share ONE GPU, so the N > 1 ncclAllGather data path runs on a
1-GPU box?

RCCL refuses two ranks of one communicator on one device ("Duplicate GPU detected")
when both ranks report the same host hash. Each rank here sets its own NCCL_HOSTID
before RCCL is loaded, so RCCL takes the ranks for separate hosts and connects them
with its network transport (sockets on lo) instead of P2P/xGMI. That is not the xGMI
path, but it is the multi-rank collective: RCCL's ring kernels, proxy threads and the
rank order of the gathered tensor.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29533 tools/probes/probe_rccl_multirank.py
"""

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
os.environ["NCCL_HOSTID"] = f"rocmdash-virt-{rank}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

dist.init_process_group("gloo")
from rocmdash.runtime import native  # noqa: E402

nat = native.load()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
lib = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
uid = nat.rccl_unique_id(lib) if rank == 0 else None
objs = [None] * world
dist.all_gather_object(objs, uid)
t0 = time.perf_counter()
comm = nat.RcclComm(0, world, rank, objs[0], lib)
init_s = time.perf_counter() - t0
x = torch.arange(16 * 8, device=dev, dtype=torch.float32).reshape(16, 8) + 1000.0 * rank
out = torch.empty((world, 16, 8), device=dev)
s = torch.cuda.current_stream(dev).cuda_stream
comm.all_gather(x.data_ptr(), out.data_ptr(), x.numel(), s)
torch.cuda.synchronize(dev)
ok = all(torch.equal(out[r], torch.arange(128, device=dev, dtype=torch.float32).reshape(16, 8) + 1000.0 * r)
         for r in range(world))
ts = []
for _ in range(200):
    t = time.perf_counter()
    comm.all_gather(x.data_ptr(), out.data_ptr(), x.numel(), s)
    torch.cuda.synchronize(dev)
    ts.append((time.perf_counter() - t) * 1e6)
dist.barrier()
res = {"rank": rank, "world": world, "ok": ok, "init_s": round(init_s, 3),
       "gather_us_p50": round(statistics.median(ts), 1), "gather_us_p90": round(sorted(ts)[180], 1)}
print(json.dumps(res), flush=True)
del comm
dist.destroy_process_group()
