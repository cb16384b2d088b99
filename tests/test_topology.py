"""HIP device order from a (fake) KFD topology: CPU nodes skipped, node-id order,
ROCR/HIP visibility index lists applied in turn, UUID lists undecidable."""

import os

import pytest

from rocmdash.runtime.topology import bdf_of_hip_device, hip_order_bdfs, kfd_gpus


def _node(root, n, simd, domain=0, loc=0):
    d = root / str(n)
    d.mkdir(parents=True)
    (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simd}\ndomain {domain}\nlocation_id {loc}\n")


@pytest.fixture
def topo(tmp_path, monkeypatch):
    for env in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(env, raising=False)
    _node(tmp_path, 0, 0)  # CPU
    _node(tmp_path, 1, 0)  # CPU
    locs = [0x8B00, 0x0A00, 0xC300, 0x2600]  # node 2..5, not in bus order
    for i, loc in enumerate(locs):
        _node(tmp_path, 2 + i, 1024, 0, loc)
    _node(tmp_path, 10, 1024, 1, 0x0500)  # second PCI domain, node id 10 sorts after 5
    return str(tmp_path), locs + [(1 << 32) | 0x0500]


def test_kfd_order(topo):
    root, bdfs = topo
    assert [b for _, b in kfd_gpus(root, check_access=False)] == bdfs
    assert hip_order_bdfs(root, check_access=False) == bdfs
    assert bdf_of_hip_device(4, root, check_access=False) == (1 << 32) | 0x0500
    assert bdf_of_hip_device(5, root, check_access=False) is None


def test_visibility_lists(topo, monkeypatch):
    root, bdfs = topo
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "3,1,2")
    assert hip_order_bdfs(root, check_access=False) == [bdfs[3], bdfs[1], bdfs[2]]
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2,0")
    assert hip_order_bdfs(root, check_access=False) == [bdfs[2], bdfs[3]]
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "GPU-abcdef")
    assert hip_order_bdfs(root, check_access=False) is None
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert hip_order_bdfs(root, check_access=False) == []


def test_missing_sysfs(tmp_path):
    assert hip_order_bdfs(str(tmp_path / "nope")) is None


@pytest.mark.gpu
def test_topology_matches_hip_on_the_box():
    """On the GPU box the sysfs walk must name the same PCI device HIP does."""
    import torch

    from rocmdash.runtime import native

    nat = native.load()
    n = torch.cuda.device_count()
    order = hip_order_bdfs()
    assert order is not None and len(order) >= n
    for i in range(n):
        assert order[i] == int(nat.hip_device_bdf(i)), (i, order, os.environ.get("HIP_VISIBLE_DEVICES"))
    # the launcher's plan on the box: one rank per physical GPU, rank r on the HIP device
    # whose PCI address the plan names
    import json
    import subprocess
    import sys

    res = subprocess.run([sys.executable, "-m", "rocmdash.launch", "--print-plan"], capture_output=True, text=True,
                         timeout=60, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    d = json.loads(res.stdout)
    print("node plan:", d)
    assert d["plan"] is not None and d["ranks"] == len(d["plan"]["gpus"]) >= 1
    for g in d["plan"]["gpus"]:
        assert g["bdf"] == int(nat.hip_device_bdf(g["hip_device"]))
    if d["plan"]["mode"] == "SPX":
        assert d["ranks"] == n and d["rank_devices"] == list(range(n))


# ---- node plan: one rank per PHYSICAL GPU, partitions grouped ----

def _tree(root, gpus, parts, uid=True, xcc_total=8):
    """A fake KFD tree: 2 CPU nodes, then ``gpus`` physical GPUs with ``parts``
    partition nodes each (same PCI address and unique_id, num_xcc split)."""
    (root / "0").mkdir(parents=True)
    (root / "0" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    (root / "1").mkdir()
    (root / "1" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    n = 2
    bdfs = []
    for g in range(gpus):
        loc = [0x0500, 0x2500, 0x4500, 0x6500, 0x8500, 0xA500, 0xC500, 0xE500][g]
        bdfs.append(loc)
        for _ in range(parts):
            d = root / str(n)
            d.mkdir()
            props = (f"cpu_cores_count 0\nsimd_count {1024 // parts}\ndomain 0\nlocation_id {loc}\n"
                     f"num_xcc {xcc_total // parts}\n")
            if uid:
                props += f"unique_id {0x1000 + g}\n"
            (d / "properties").write_text(props)
            n += 1
    return str(root), bdfs


@pytest.fixture
def clean_env(monkeypatch):
    for env in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCMDASH_RANK_DEVICES",
                "ROCMDASH_OVERSUBSCRIBE"):
        monkeypatch.delenv(env, raising=False)


@pytest.mark.parametrize("gpus,parts,mode", [(8, 1, "SPX"), (8, 8, "CPX"), (4, 1, "SPX"), (8, 2, "DPX"),
                                             (1, 4, "QPX")])
@pytest.mark.parametrize("uid", [True, False])
def test_node_plan_one_rank_per_physical_gpu(tmp_path, clean_env, gpus, parts, mode, uid):
    from rocmdash.runtime.topology import node_plan, rank_devices

    root, bdfs = _tree(tmp_path, gpus, parts, uid)
    plan = node_plan(root, check_access=False)
    assert plan["mode"] == mode and plan["logical_devices"] == gpus * parts
    assert len(plan["gpus"]) == gpus  # ranks = physical GPUs (8 x CPX: 64 devices, 8 ranks)
    for r, g in enumerate(plan["gpus"]):
        assert g["rank"] == r and g["bdf"] == bdfs[r]
        assert g["partitions"] == list(range(r * parts, (r + 1) * parts)) and g["hip_device"] == r * parts
        assert g["num_xcc"] == 8  # every XCD of the GPU belongs to exactly one rank
    assert rank_devices(plan) == [r * parts for r in range(gpus)]


def test_node_plan_follows_visibility(tmp_path, clean_env, monkeypatch):
    """Visible devices 8..15 (the second GPU's CPX partitions) and 0: two physical GPUs,
    HIP indices renumbered."""
    from rocmdash.runtime.topology import node_plan

    root, bdfs = _tree(tmp_path, 8, 8)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", ",".join(map(str, list(range(8, 16)) + [0])))
    plan = node_plan(root, check_access=False)
    assert [g["bdf"] for g in plan["gpus"]] == [bdfs[1], bdfs[0]]
    assert plan["gpus"][0]["partitions"] == list(range(8)) and plan["gpus"][1]["partitions"] == [8]
    assert plan["mode"] == "mixed"
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "GPU-1234")
    assert node_plan(root, check_access=False) is None


def test_rank_devices_env_and_partitioned_nodes(tmp_path, clean_env, monkeypatch):
    from rocmdash.parallel import node
    from rocmdash.runtime import topology

    import torch

    root, _ = _tree(tmp_path, 8, 8)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 64)  # HIP sees every partition
    monkeypatch.setattr(topology, "KFD_NODES", root)
    real = topology.node_plan
    monkeypatch.setattr(topology, "node_plan", lambda r=root, check_access=False: real(r, check_access=False))
    assert [node.device_index_for(r) for r in range(8)] == [8 * r for r in range(8)]
    monkeypatch.setenv("ROCMDASH_RANK_DEVICES", "3,1")
    assert node.device_index_for(0) == 3 and node.device_index_for(1) == 1
    monkeypatch.delenv("ROCMDASH_RANK_DEVICES")
    root1, _ = _tree(tmp_path / "spx", 8, 1)
    monkeypatch.setattr(topology, "node_plan", lambda r=root1, check_access=False: real(r, check_access=False))
    assert [node.device_index_for(r) for r in range(8)] == list(range(8))  # SPX: the local rank
    monkeypatch.setattr(topology, "node_plan", lambda r=root, check_access=False: real(r, check_access=False))
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)  # KFD lists GPUs HIP cannot use: no plan
    assert node.device_index_for(1) == 1


@pytest.mark.parametrize("gpus,parts", [(8, 1), (8, 8), (4, 1)])
def test_launch_starts_one_rank_per_physical_gpu(tmp_path, clean_env, monkeypatch, gpus, parts):
    import torch

    from rocmdash import launch

    monkeypatch.setattr(torch.cuda, "device_count", lambda: gpus * parts)
    root, _ = _tree(tmp_path, gpus, parts)
    import rocmdash.runtime.topology as topology

    real = topology.node_plan
    try:
        topology.node_plan = lambda r=None, check_access=True: real(root, check_access=False)
        n, devices, plan = launch.plan_ranks("auto")
    finally:
        topology.node_plan = real
    assert n == gpus and devices == [r * parts for r in range(gpus)]
    assert launch.plan_ranks("3")[0] == 3
    # a container whose KFD tree lists GPUs HIP cannot open: one rank per HIP device
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    try:
        topology.node_plan = lambda r=None, check_access=True: real(root, check_access=False)
        assert launch.plan_ranks("auto")[:2] == (1, None)
    finally:
        topology.node_plan = real


def test_launch_supervises_the_service_cpu():
    """``python -m rocmdash.launch`` (default: supervised) starts one rank per slot: 2 CPU
    service ranks form epoch 1, run 3 refreshes, vote to stop together, and the
    supervisor exits 0 without restarting them (a stop vote is not a failure)."""
    import socket
    import subprocess
    import sys

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    res = subprocess.run([sys.executable, "-m", "rocmdash.launch", "--nproc", "2", f"--master-port={port}",
                          "-m", "rocmdash.serve", "--cpu", "--source", "synthetic", "--counters", "synthetic",
                          "--port", "0", "--refresh-hz", "20", "--max-refreshes", "3"],
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), capture_output=True, text=True,
                         timeout=180, env=env)
    out = res.stdout + res.stderr
    assert res.returncode == 0, out[-4000:]
    assert "[rocmdash.launch] supervising 2 rank(s)" in out and "epoch 1: members [0, 1]" in out, out[-4000:]
    assert "slot 0 stopped after 3 refreshes" in out and "slot 1 stopped after 3 refreshes" in out, out[-4000:]
    assert "started incarnation 1" not in out


def test_launch_runs_the_service_cpu(tmp_path):
    """``python -m rocmdash.launch --torchrun`` starts torchrun as a child with the rank
    count and forwards the rest: 2 CPU service ranks run 3 refreshes and every process
    exits 0."""
    import socket
    import subprocess
    import sys

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    res = subprocess.run([sys.executable, "-m", "rocmdash.launch", "--torchrun", "--nproc", "2", "--master-addr", "127.0.0.1",
                          "--master-port", str(port), "-m", "rocmdash.serve", "--cpu", "--source", "synthetic",
                          "--counters", "synthetic", "--port", "0", "--refresh-hz", "20", "--max-refreshes", "3"],
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), capture_output=True, text=True,
                         timeout=180, env=env)
    out = res.stdout + res.stderr
    assert res.returncode == 0, out[-4000:]
    assert "[rocmdash.launch] 2 rank(s)" in out and "--nproc-per-node=2" in out
    assert "rank 0 stopped after 3 refreshes (exit 0)" in out and "rank 1 stopped after 3 refreshes (exit 0)" in out
