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
