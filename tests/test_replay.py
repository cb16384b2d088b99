"""Replay of a telemetry capture recorded on a real MI355X (tests/fixtures/, made with
``python -m rocmdash.runtime.record --load`` on the GPU box): the whole CPU pipeline
runs on hardware-shaped data - rings, window statistics (numpy reference of the
kernel), node snapshot and the dashboard frame - and the values stay physical."""

import json
import os

import numpy as np
import pytest

from rocmdash.config import SamplerConfig
from rocmdash.models.schema import CTR_FIELDS, SMI_FIELDS
from rocmdash.ops.window_stats import window_stats_reference
from rocmdash.runtime.record import load_recording, record

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "mi355x_capture.npz")


@pytest.fixture(scope="module")
def capture():
    if not os.path.exists(FIXTURE):
        pytest.skip("no MI355X capture in tests/fixtures (record one with tools/gpu_round.sh record)")
    return load_recording(FIXTURE)


def test_capture_is_physical(capture):
    info = capture["info"]
    assert info["card_model"].startswith("102-") and "MI355" in info["product_name"]
    smi = capture["smi_rows"]
    assert smi.shape[1] == len(SMI_FIELDS) and len(smi) >= 100
    c = {n: smi[:, i] for i, n in enumerate(SMI_FIELDS)}
    assert np.nanmin(c["amd_gpu_edge_temperature"]) > 10 and np.nanmax(c["amd_gpu_edge_temperature"]) < 120
    assert np.nanmax(c["amd_gpu_average_package_power"]) < 2000 and np.nanmin(c["amd_gpu_average_package_power"]) > 50
    assert np.nanmax(c["amd_gpu_gfx_activity"]) <= 100
    assert np.all(c["amd_gpu_total_vram"] > 200_000)
    if "counter_rows" in capture:
        ctr = capture["counter_rows"]
        k = {n: ctr[:, i] for i, n in enumerate(CTR_FIELDS)}
        assert np.nanmax(k["amd_gpu_mfma_utilization"]) > 5  # recorded under a bf16 GEMM load
        assert np.nanmax(k["amd_gpu_hbm_read_bandwidth"]) > 1


def test_replay_drives_the_pipeline(capture):
    from rocmdash.parallel.node import NodeAggregator
    from rocmdash.runtime.agent import GpuAgent
    from rocmdash.runtime.pipeline import NodePipeline

    n = len(capture["smi_rows"])
    agent = GpuAgent(0, source="replay", replay=capture, cfg=SamplerConfig(window=256, ring_capacity=1024),
                     use_gpu=False)
    assert agent.info.smi_backend == "replay"
    agent.prefill(min(n, 300))
    pipe = NodePipeline(agent, NodeAggregator(), extended=True)
    payload, _ = pipe.step()
    d = json.loads(payload)
    assert d["headers"] == ["### GPU 0 (MI355X)"]
    rows, _ = agent.smi_ring.window(256)
    ref = window_stats_reference(rows.T)
    np.testing.assert_allclose(agent.refresh().numpy()[: len(SMI_FIELDS)], ref, rtol=1e-5)
    # the replayed rows are the recorded ones, in order (300 prefill samples + the step's)
    np.testing.assert_array_equal(rows[-1], capture["smi_rows"][300 % n])


def test_record_roundtrip(tmp_path):
    from rocmdash.runtime.agent import GpuAgent

    a = GpuAgent(0, source="synthetic", counters="synthetic", cfg=SamplerConfig(window=64, ring_capacity=256),
                 use_gpu=False)
    a.prefill(100)
    rec = record(a, str(tmp_path / "r.npz"))
    back = load_recording(str(tmp_path / "r.npz"))
    np.testing.assert_array_equal(back["smi_rows"], rec["smi_rows"])
    np.testing.assert_array_equal(back["counter_ts"], rec["counter_ts"])
    assert back["info"]["series"] == list(SMI_FIELDS + CTR_FIELDS)
    b = GpuAgent(0, source="replay", replay=str(tmp_path / "r.npz"), cfg=SamplerConfig(window=64, ring_capacity=256),
                 use_gpu=False)
    b.prefill(100)
    np.testing.assert_array_equal(b.smi_ring.window(100)[0], rec["smi_rows"])


def test_old_capture_layout_replays_with_nan_columns(tmp_path):
    """A capture made before series were added (8 SMI columns) loads onto the current
    layout by series name: the new columns replay as NaN (skipped by the statistics)."""
    from rocmdash.runtime.agent import GpuAgent
    from rocmdash.runtime.record import upgrade_layout

    old_smi = [n for n in SMI_FIELDS if "xgmi" not in n and "pcie" not in n]
    assert len(old_smi) == 8
    rows = np.arange(5 * 8, dtype=np.float32).reshape(5, 8)
    rec = {"info": {"series": old_smi + list(CTR_FIELDS)}, "smi_rows": rows,
           "counter_rows": np.ones((5, len(CTR_FIELDS)), np.float32)}
    up = upgrade_layout(rec)
    assert up["smi_rows"].shape == (5, len(SMI_FIELDS))
    for j, name in enumerate(old_smi):
        np.testing.assert_array_equal(up["smi_rows"][:, SMI_FIELDS.index(name)], rows[:, j])
    new = [SMI_FIELDS.index(n) for n in SMI_FIELDS if n not in old_smi]
    assert np.isnan(up["smi_rows"][:, new]).all()
    assert up["info"]["series"] == list(SMI_FIELDS + CTR_FIELDS)
    a = GpuAgent(0, source="replay", replay=up, cfg=SamplerConfig(window=64, ring_capacity=256), use_gpu=False)
    a.prefill(5)
    st = a.refresh().numpy()
    assert st[new, 7].tolist() == [0.0] * len(new)  # count of valid samples
