"""Native runtime on the CPU: SPSC ring semantics (window, wrap, torn reads), the
sampler thread (rate, stats, SPSC guard), synthetic sources, the CPU path of the
agent and the numpy reference of the window-stats kernel."""

import threading
import time

import numpy as np
import pytest

from rocmdash.models.schema import CTR_FIELDS, SMI_FIELDS
from rocmdash.ops.window_stats import window_stats_reference
from rocmdash.viz.panels import EXTENDED_PANELS


def test_layout_matches_schema(native):
    assert tuple(native.SMI_FIELDS) == SMI_FIELDS and tuple(native.CTR_FIELDS) == CTR_FIELDS


def test_ring_push_window_wrap(native):
    r = native.SeriesRing(3, 8)
    assert r.head == 0 and r.window(4)[0].shape == (0, 3)
    for i in range(21):
        r.push(np.array([i, 2 * i, -i], np.float32), 1000 + i)
    assert r.head == 21 and r.last_timestamp == 1020
    rows, ts = r.window(5)
    np.testing.assert_array_equal(rows[:, 0], np.arange(16, 21))
    np.testing.assert_array_equal(ts, 1000 + np.arange(16, 21))
    rows, _ = r.window(100)  # clipped to capacity
    np.testing.assert_array_equal(rows[:, 0], np.arange(13, 21))


def test_ring_rejects_bad_shapes(native):
    with pytest.raises(Exception):
        native.SeriesRing(3, 6)  # not a power of two
    with pytest.raises(Exception):
        native.SeriesRing(0, 8)
    r = native.SeriesRing(2, 4)
    with pytest.raises(Exception):
        r.push(np.zeros(3, np.float32), 0)


def test_ring_push_many(native):
    r = native.SeriesRing(2, 16)
    rows = np.arange(20, dtype=np.float32).reshape(10, 2)
    r.push_many(rows, np.arange(10, dtype=np.uint64))
    got, ts = r.window(10)
    np.testing.assert_array_equal(got, rows)


def test_ring_concurrent_reader_never_sees_torn_rows(native):
    """Producer thread (native sampler) vs Python reader: every row read must be
    internally consistent (all columns from the same push)."""
    src = native.make_synthetic_source("smi", 1)
    r = native.SeriesRing(src.width, 64)
    s = native.Sampler(src, r, 20000.0)
    s.start()
    try:
        deadline = time.time() + 1.0
        reads = 0
        while time.time() < deadline:
            rows, ts = r.window(64)
            if len(rows):
                # total VRAM column is constant, used <= total, temps equal (hotspot mirrors edge)
                assert np.all(rows[:, 4] == rows[0, 4])
                np.testing.assert_array_equal(rows[:, 0], rows[:, 5])
                assert np.all(np.diff(ts.astype(np.int64)) >= 0)
                reads += 1
        assert reads > 10
    finally:
        s.stop()
    assert s.stats()["samples"] > 100


def test_sampler_rate_and_stats(native):
    r = native.SeriesRing(len(native.CTR_FIELDS), 1024)
    s = native.Sampler(native.make_synthetic_source("counter", 2), r, 200.0)
    s.start()
    time.sleep(0.5)
    s.stop()
    n = s.stats()["samples"]
    assert 60 <= n <= 140, n  # ~100 at 200 Hz over 0.5 s
    assert not s.running
    assert s.sample_once() is True


def test_sample_once_refused_while_running(native):
    r = native.SeriesRing(len(native.CTR_FIELDS), 64)
    s = native.Sampler(native.make_synthetic_source("counter", 2), r, 50.0)
    s.start()
    try:
        with pytest.raises(RuntimeError):
            s.sample_once()
    finally:
        s.stop()


def test_sampler_width_mismatch(native):
    with pytest.raises(Exception):
        native.Sampler(native.make_synthetic_source("smi", 1), native.SeriesRing(3, 8), 10.0)


def test_synthetic_sources_deterministic_and_plausible(native):
    a = native.make_synthetic_source("smi", 7)
    b = native.make_synthetic_source("smi", 7)
    ra = np.stack([a.sample() for _ in range(200)])
    rb = np.stack([b.sample() for _ in range(200)])
    np.testing.assert_array_equal(ra, rb)
    assert np.all((ra[:, 1] >= 0) & (ra[:, 1] <= 100))
    assert np.all(ra[:, 3] <= ra[:, 4])
    assert a.info()["model_number"] == "102-G36236-0C"
    c = native.make_synthetic_source("counter", 7)
    rc = np.stack([c.sample() for _ in range(200)])
    assert np.all((rc[:, 0] >= 0) & (rc[:, 0] <= 100)) and np.all(rc[:, 1] >= 0)
    with pytest.raises(Exception):
        native.make_synthetic_source("nope", 1)


def test_synthetic_xcd_detail(native):
    """Per-XCD busy / clocks: none before the first sample, eight of each after, and the
    row streams are the same whether or not the detail is read."""
    a = native.make_synthetic_source("smi", 3)
    assert a.xcd_detail() is None
    a.sample()
    d = a.xcd_detail()
    assert d["busy"].shape == (8,) and d["clock_mhz"].shape == (8,)
    assert np.all((d["busy"] >= 0) & (d["busy"] <= 100)) and np.all((d["clock_mhz"] > 1000) & (d["clock_mhz"] < 2500))
    b = native.make_synthetic_source("smi", 3)
    b.sample()
    np.testing.assert_array_equal(a.sample(), b.sample())
    assert native.make_synthetic_source("counter", 3).xcd_detail() is None


def test_window_stats_reference_matches_numpy():
    rng = np.random.default_rng(0)
    x = rng.normal(size=(5, 301))
    x[1, ::4] = np.nan
    x[2] = np.nan
    out = window_stats_reference(x)
    v = x[0]
    np.testing.assert_allclose(out[0, :6], [v.min(), v.max(), v.mean(), *np.percentile(v, [50, 90, 99])])
    assert out[0, 6] == x[0, -1] and out[0, 7] == 301
    assert out[2, 7] == 0 and np.isnan(out[2, :7]).all()
    assert out[1, 7] == 301 - 76


def test_window_stats_torch_reference_matches_numpy():
    torch = pytest.importorskip("torch")
    from rocmdash.ops.window_stats import window_stats_torch

    rng = np.random.default_rng(1)
    x = rng.normal(size=(4, 257)).astype(np.float32)
    x[3, ::2] = np.nan
    a = window_stats_torch(torch.from_numpy(x)).numpy()
    b = window_stats_reference(x)
    np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6)


def test_cpu_agent_refresh(native):
    from rocmdash.config import SamplerConfig
    from rocmdash.runtime.agent import GpuAgent

    agent = GpuAgent(0, source="synthetic", counters="synthetic", cfg=SamplerConfig(window=128, ring_capacity=512),
                     use_gpu=False)
    agent.prefill(200)
    out = agent.refresh().numpy()
    rows, _ = agent.smi_ring.window(128)
    np.testing.assert_allclose(out[: len(SMI_FIELDS)], window_stats_reference(rows.T), rtol=1e-5)
    assert agent.series == SMI_FIELDS + CTR_FIELDS
    assert agent.info.smi_backend == "synthetic" and agent.info.counter_backend == "synthetic"
    x = agent.xcd()
    assert x.shape == (2, 8) and np.isfinite(x).all()
    agent.close()


def test_cpu_pipeline_world1(native):
    import json

    from rocmdash.config import SamplerConfig
    from rocmdash.parallel.node import NodeAggregator
    from rocmdash.runtime.agent import GpuAgent
    from rocmdash.runtime.pipeline import NodePipeline

    agent = GpuAgent(0, source="synthetic", counters="synthetic", cfg=SamplerConfig(window=64, ring_capacity=256),
                     use_gpu=False)
    agent.prefill(64)
    pipe = NodePipeline(agent, NodeAggregator(), extended=True)
    payload, tm = pipe.step()
    d = json.loads(payload)
    assert len(d["figures"]) == 4 + 4 + len(EXTENDED_PANELS)
    assert d["window"]["gpus"] == ["0"] and d["window"]["series"] == list(agent.series)
    assert len(d["window"]["values"][0]) == len(agent.series)
    assert tm.total_ms > 0
    snap = pipe.latest_snapshot()
    assert snap.has("amd_gpu_mfma_utilization") and snap.has("vram_usage_ratio")


def test_background_agent_sampling(native):
    from rocmdash.config import SamplerConfig
    from rocmdash.runtime.agent import GpuAgent

    agent = GpuAgent(0, source="synthetic", counters="synthetic",
                     cfg=SamplerConfig(window=64, ring_capacity=256, smi_hz=100, counter_hz=400), use_gpu=False)
    agent.start()
    time.sleep(0.3)
    agent.stop()
    st = agent.sampler_stats()
    assert st[0]["samples"] >= 15 and st[1]["samples"] >= 60
    assert agent.smi_ring.head == st[0]["samples"]
    assert threading.active_count() >= 1


def test_sampler_single_producer_guards(native):
    """The ring is SPSC: a pending request() blocks start() and sample_once() until
    wait() (the advisor's round-1 finding), and counts() is the cheap stats read."""
    r = native.SeriesRing(len(native.CTR_FIELDS), 64)
    s = native.Sampler(native.make_synthetic_source("counter", 2), r, 50.0)
    s.request()
    with pytest.raises(RuntimeError):
        s.sample_once()
    with pytest.raises(RuntimeError):
        s.start()
    assert s.wait() is True
    assert s.sample_once() is True
    assert s.counts() == (2, 0, 0)
    s.start()
    try:
        with pytest.raises(RuntimeError):
            s.request()
    finally:
        s.stop()


def test_free_running_sampler_calls_and_rate_cap(native):
    """start_free(): back-to-back reads on the background thread, starts at most max_hz
    apart; calls() / last_start_ns() / wait_calls() let a refresh wait for a new row
    (perf_counter clock); stop() returns the sampler to paced / closed-loop use."""
    r = native.SeriesRing(len(native.CTR_FIELDS), 4096)
    s = native.Sampler(native.make_synthetic_source("counter", 3), r, 10.0)
    assert s.calls() == 0 and list(s.recent_us()) == []
    s.start_free(2000.0)
    try:
        with pytest.raises(RuntimeError):
            s.start_free(2000.0)
        c0 = s.calls()
        c1 = s.wait_calls(c0 + 5, 2.0)
        assert c1 >= c0 + 5
        age = time.perf_counter_ns() - s.last_start_ns()
        assert -5e6 < age < 1e8  # same clock as time.perf_counter_ns
        time.sleep(0.25)
    finally:
        s.stop()
    n = s.calls()
    assert 200 <= n <= 2000 * 0.3 + 10  # capped at 2 kHz, far above the 10 Hz pacing
    assert s.counts()[0] == n == r.head
    assert len(s.recent_us()) == min(n, 1024)
    assert s.wait_calls(n + 1, 0.01) == n  # nothing running: times out, returns the count
    assert s.sample_once() is True  # closed-loop use again


def test_free_running_pipeline_reduces_every_new_row(native):
    """NodePipeline(sampling="free"): each refresh waits until every source has at least
    one new row since the previous refresh (the reads themselves never wait for a
    refresh); stop_sampling() hands the agent back to closed loop."""
    from rocmdash.config import SamplerConfig
    from rocmdash.parallel.node import NodeAggregator
    from rocmdash.runtime.agent import GpuAgent
    from rocmdash.runtime.pipeline import NodePipeline

    agent = GpuAgent(0, source="synthetic", counters="synthetic", cfg=SamplerConfig(window=64, ring_capacity=1024),
                     use_gpu=False)
    agent.prefill(64)
    pipe = NodePipeline(agent, NodeAggregator(), sampling="free")
    c0 = agent.sample_counts()
    pipe.start_sampling()
    try:
        for _ in range(20):
            before = list(pipe._free_calls)  # the counts the previous refresh saw
            t0, t1 = pipe.sample_phase()
            assert all(now > b for now, b in zip(pipe._free_calls, before))
            assert t0 <= t1
            pipe.gather()
    finally:
        pipe.stop_sampling()
    c1 = agent.sample_counts()
    assert c1["counter_rows"] - c0["counter_rows"] >= 20 and c1["smi_rows"] - c0["smi_rows"] >= 20
    assert not any(s.running for s in agent.samplers)
    agent.sample()  # closed loop works again
    agent.close()


@pytest.mark.parametrize("sampling", ["closed", "free"])
def test_bench_counts_only_reads_inside_the_timed_window(native, sampling):
    """bench.py's accounting in both sampling modes (CPU, synthetic sources: every row
    is fresh, 15 fresh series per row pair): closed loop counts exactly K reads per
    source for K steps; free-running counts the rows completed between t0 and t1 -
    never fewer than one per source per step, never more than the rate cap allows."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    K = 40
    res = subprocess.run([sys.executable, "bench.py", "--cpu", "--steps", str(K), "--warmup", "3", "--window", "128",
                          "--e2e-s", "0", "--sampling", sampling], cwd=root, capture_output=True, text=True,
                         timeout=120, env=dict(os.environ, ROCMDASH_FREE_MAX_HZ="20000"))
    assert res.returncode == 0, res.stderr[-3000:]
    d = json.loads(res.stdout.strip().splitlines()[-1])
    assert d["sampling"] == sampling
    per_row = 15  # 5 counter deltas + used VRAM + 9 SMU-table series (synthetic: all new)
    if sampling == "closed":
        assert d["fresh_samples"] == K * per_row
    else:
        assert d["fresh_samples"] >= (K - 1) * per_row  # the first step may take a row from before t0
        timed_s = d["ranks"][0]["timed_s"]
        assert d["fresh_samples"] <= (20000 * timed_s + 2) * per_row


def test_fresh_sample_accounting(native):
    """bench.py's fresh count: counter rows x 5, used VRAM per SMI row, SMU-table
    series only per table publication (synthetic sources: every row is new)."""
    from rocmdash.config import SamplerConfig
    from rocmdash.models.schema import CTR_FIELDS, SMI_TABLE_FIELDS
    from rocmdash.runtime.agent import GpuAgent

    a = GpuAgent(0, source="synthetic", counters="synthetic", cfg=SamplerConfig(window=64, ring_capacity=256),
                 use_gpu=False)
    c0 = a.sample_counts()
    for _ in range(10):
        a.sample()
    c1 = a.sample_counts()
    assert c1["smi_rows"] - c0["smi_rows"] == 10 and c1["counter_rows"] - c0["counter_rows"] == 10
    assert a.fresh_samples(c0, c1) == 10 * (len(CTR_FIELDS) + 1 + len(SMI_TABLE_FIELDS))
    # a hardware SMI source that saw 2 table publications over 10 reads
    hw0 = dict(c0, smi_table_changes=5)
    hw1 = dict(c1, smi_table_changes=7)
    assert a.fresh_samples(hw0, hw1) == 10 * len(CTR_FIELDS) + 10 + 2 * len(SMI_TABLE_FIELDS)
    assert a.fresh_breakdown(hw0, hw1) == {"counters": 10 * len(CTR_FIELDS), "used_vram": 10,
                                           "smu_table": 2 * len(SMI_TABLE_FIELDS)}
    a.close()


def test_health_rows_and_source_health(native):
    import numpy as np

    from rocmdash.config import SamplerConfig
    from rocmdash.models.health import SourceHealth
    from rocmdash.models.schema import HEALTH_INDEX
    from rocmdash.runtime.agent import GpuAgent

    a = GpuAgent(0, source="synthetic", counters="synthetic", cfg=SamplerConfig(window=64, ring_capacity=256),
                 use_gpu=False)
    for _ in range(3):
        a.sample()
    rows = a.health_rows(np.empty((2, 8), np.float32))
    assert rows[0, HEALTH_INDEX["samples_lo"]] == 3 and rows[1, HEALTH_INDEX["samples_lo"]] == 3
    assert rows[0, HEALTH_INDEX["hz"]] == a.cfg.smi_hz and rows[1, HEALTH_INDEX["present"]] == 1
    h = SourceHealth(rows[None], [("synthetic", "synthetic")])
    st = h.statuses()
    assert [s.kind for s in st] == ["smi", "counter"] and not any(s.stale for s in st)
    # far in the future: both sources are stale
    late = a.health_rows(np.empty((2, 8), np.float32), now_ns=time.time_ns() + int(60e9))
    assert SourceHealth(late[None], [("s", "c")]).stale_gpus() == [0]
    # counts above 2^24 survive the float32 split exactly
    big = rows.copy()
    big[0, HEALTH_INDEX["samples_hi"]], big[0, HEALTH_INDEX["samples_lo"]] = divmod(123_456_789_012, 1 << 24)
    assert SourceHealth(big[None], [("s", "c")]).statuses()[0].samples == 123_456_789_012
    a.close()
