"""Long-window statistics (csrc/long_window.hip): HBM-resident windows beyond LDS
capacity, exact percentiles by a multi-workgroup radix select, against the fp64 numpy
reference over the same rows - ties, NaN, constant and signed-zero series, device-ring
wrap-around, host-ring overflow (lost rows become NaN), graph vs direct launches."""

import numpy as np
import pytest

from rocmdash.ops.window_stats import window_stats_reference

pytestmark = pytest.mark.gpu


def _rows(rng, k, width, base):
    x = rng.integers(0, 50, size=(k, width)).astype(np.float32)  # telemetry-like ties
    x[:, 0] = rng.normal(100, 20, k)  # continuous
    if width > 2:
        x[:, 1] = 42.0  # constant
    if width > 3:
        x[:, 2] = rng.choice(np.array([-0.0, 0.0, -1.5, 3.25], np.float32), k)  # signed zeros
    x[rng.random((k, width)) < 0.05] = np.nan
    x[:, -1] = base + np.arange(k, dtype=np.float32)  # monotone: ordering / last
    return x


class _Mirror:
    """Everything pushed, oldest first; lost rows are NaN."""

    def __init__(self, width):
        self.rows = np.zeros((0, width), np.float32)

    def push(self, x):
        self.rows = np.concatenate([self.rows, x])

    def lose(self, lo, hi):
        self.rows[lo:hi] = np.nan

    def window(self, W):
        return self.rows[-W:]


def _check(out, mirrors, W):
    ref = np.concatenate([window_stats_reference(m.window(W).T) for m in mirrors])
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("W", [1024, 65536, 1 << 20])
def test_long_window_matches_reference(native, cuda, W):
    import torch

    nat = native
    nat.set_pinned_host_rings(True)
    cap = 1 << 17
    ra, rb = nat.SeriesRing(8, cap), nat.SeriesRing(4, cap)
    lw = nat.LongWindowSet(W, 0, use_graph=True)
    lw_direct = nat.LongWindowSet(W, 0)  # the default: direct launches
    # the smallest chunk: 16x the workgroups of the default at W = 2^20 (exact ranks, the
    # mean only summed in another order)
    lw_small = nat.LongWindowSet(W, 0, chunk_rows=256)
    for s in (lw, lw_direct, lw_small):
        s.add_ring(ra)
        s.add_ring(rb)
    ma, mb = _Mirror(8), _Mirror(4)
    out = torch.empty((12, 8), device=cuda)
    out2 = torch.empty((12, 8), device=cuda)
    out3 = torch.empty((12, 8), device=cuda)
    rng = np.random.default_rng(W)
    t = 0
    # every push fits the host ring (cap) so nothing is lost between refreshes
    steps = [min(cap, W // 3 + 5), 1, 0, 7, min(cap, W), 3, min(cap - 1, W + 11), 1]
    while sum(steps) < W + 3:
        steps.append(min(cap, W))
    for k in steps:
        xa, xb = _rows(rng, k, 8, t), _rows(rng, k, 4, -t)
        ra.push_many(xa, np.arange(t, t + k, dtype=np.uint64))
        rb.push_many(xb, np.arange(t, t + k, dtype=np.uint64))
        ma.push(xa)
        mb.push(xb)
        t += k
        stream = torch.cuda.current_stream().cuda_stream
        lw.refresh(out.data_ptr(), stream)
        lw_direct.refresh(out2.data_ptr(), stream)
        lw_small.refresh(out3.data_ptr(), stream)
        torch.cuda.synchronize()
        _check(out, [ma, mb], W)
        _check(out3, [ma, mb], W)
        # graph and direct launches compute the same bits (fixed reduction order)
        assert torch.equal(out.nan_to_num(-7.0), out2.nan_to_num(-7.0))
        # other chunking: every order statistic identical
        keep = [0, 1, 3, 4, 5, 6, 7]
        assert torch.equal(out[:, keep].nan_to_num(-7.0), out3[:, keep].nan_to_num(-7.0))
    assert lw.chunk_rows >= 256 and lw_small.chunk_rows == 256
    # the default plans each ring's chunk by its row bytes (non-power-of-two rows at 2^20)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert lw_direct.chunk_plan == nat.long_window_chunk_plan(W, [8, 4], cus, 0, lw_direct.plan_rounds)
    assert lw_small.chunk_plan == [(256, W // 256)] * 2
    if W == 1 << 20:  # one round: balanced by bytes (non-power-of-two rows); more: equal rows
        one = nat.long_window_chunk_plan(W, [8, 4], cus)
        assert one[0][0] < one[1][0], one
        if lw_direct.plan_rounds > 1:
            assert lw_direct.chunk_plan[0][0] == lw_direct.chunk_plan[1][0], lw_direct.chunk_plan
    st = lw.stats()
    assert st["graph_launches"] == len(steps) and st["rows_lost"] == 0
    # incremental bracket mode (direct launches): pass B + scan B (whose last workgroup
    # writes the report) on the refreshes whose series want brackets (none before the
    # first refresh's scan 3 says so) - ONE kernel when scan B streams a short work list
    # itself (fused) -, the radix chain's 8 kernels only on the refreshes the brackets left
    # series to
    sd = lw_direct.stats()
    assert sd["kernel_launches"] == (8 * sd["chain_refreshes"] + 2 * sd["bracket_refreshes"]
                                     - sd["single_kernel_refreshes"]), sd
    assert 0 < sd["bracket_refreshes"] < len(steps) and sd["chain_refreshes"] <= len(steps)


def test_long_window_lost_rows_and_percentiles(native, cuda):
    """Rows the host ring overwrote before a refresh are NaN in the window; other
    percentiles than the defaults."""
    import torch

    nat = native
    nat.set_pinned_host_rings(True)
    W, cap = 1 << 16, 1 << 12
    ring = nat.SeriesRing(8, cap)
    lw = nat.LongWindowSet(W, 0)
    lw.add_ring(ring)
    m = _Mirror(8)
    out = torch.empty((8, 8), device=cuda)
    rng = np.random.default_rng(3)
    t = 0
    for k, refresh in [(3000, True), (3 * cap + 100, True), (cap, True), (10, True)]:
        x = _rows(rng, k, 8, t)
        ring.push_many(x, np.arange(t, t + k, dtype=np.uint64))
        before = len(m.rows)
        m.push(x)
        lost = max(0, k - cap)
        if lost:
            m.lose(before, before + lost)
        t += k
        lw.refresh(out.data_ptr(), torch.cuda.current_stream().cuda_stream, 5.0, 25.0, 75.0)
        torch.cuda.synchronize()
        ref = window_stats_reference(m.window(W).T, (5.0, 25.0, 75.0))
        np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-4)
    assert lw.stats()["rows_lost"] == 2 * cap + 100


def test_agent_uses_long_window_beyond_lds(native, cuda):
    from rocmdash.config import SamplerConfig
    from rocmdash.runtime.agent import GpuAgent

    cfg = SamplerConfig(window=1 << 16, ring_capacity=1 << 16)
    a = GpuAgent(0, source="synthetic", counters="synthetic", cfg=cfg)
    assert type(a.dws).__name__ == "LongWindowSet"
    a.prefill(70000)
    got = a.refresh().cpu().numpy()
    ref = np.concatenate([window_stats_reference(r.window(1 << 16)[0].T) for r in a.rings])
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-4)
    a.close()


def test_long_window_adaptive_digits_follow_the_range(native, cuda):
    """Pass 0 predicts the key bits that vary from the previous window's min / max and the
    rows that entered since (<= 256: else no prediction), and the passes stop at the lowest
    bit any sample varies in; bracket mode resolves a series in one pass when its
    percentiles stay inside the previous refresh's brackets, else the radix chain does. Windows whose range grows (spikes, a monotone series, a
    constant that changes) and shrinks (spikes leaving), mixed signs, tiny and huge
    magnitudes, all-NaN stretches, refreshes with 0..256 and more new rows: every
    refresh exact against the fp64 reference, graph == direct launches. Rings of 16 and
    13 series are streamed as two segments of <= 8 (13: unaligned rows, scalar loads)."""
    import torch

    nat = native
    nat.set_pinned_host_rings(True)
    W, cap = 2048, 1 << 14
    ring, r16, r13 = nat.SeriesRing(6, cap), nat.SeriesRing(16, cap), nat.SeriesRing(13, cap)
    lw, lwg = nat.LongWindowSet(W, 0), nat.LongWindowSet(W, 0, use_graph=True)
    # the pre-round-4 kernels: one shared pass-0 LDS histogram, pass 3 streaming the
    # window (no candidate compaction); and the next-rows prefetch modes - the same order
    # statistics
    lwo = nat.LongWindowSet(W, 0)
    lwo.wave_private = False
    lwo.compact = False
    lwo.prefetch = 2
    lwo.incremental = False  # bracket mode streaming every chunk, re-centred every hit
    lwp = nat.LongWindowSet(W, 0)
    lwp.prefetch = 1
    lwp.compact = True  # candidate compaction (pass 2 -> pass 3)
    lwr = nat.LongWindowSet(W, 0)  # the radix chain alone (no bracket mode)
    lwr.brackets = False
    lwr.wave_private_level = 2  # and pass 0's LDS copies per half wave
    lwu = nat.LongWindowSet(W, 0)  # incremental pass B always its own kernel (never fused into scan B)
    lwu.fused_passb = False
    assert not lw.compact and lw.wave_private and lw.prefetch == 0 and lw.brackets and lw.incremental
    assert lw.fused_passb
    for s in (lw, lwg, lwo, lwp, lwr, lwu):
        for r in (ring, r16, r13):
            s.add_ring(r)
    m, m16, m13 = _Mirror(6), _Mirror(16), _Mirror(13)
    out, outg = torch.empty((35, 8), device=cuda), torch.empty((35, 8), device=cuda)
    outo, outp = torch.empty((35, 8), device=cuda), torch.empty((35, 8), device=cuda)
    outr, outu = torch.empty((35, 8), device=cuda), torch.empty((35, 8), device=cuda)
    rng = np.random.default_rng(11)
    t = 0
    steps = [300] + list(rng.choice([0, 1, 2, 5, 64, 200, 256, 257, 700], size=48))
    for i, k in enumerate(steps):
        k = int(k)
        x = np.empty((k, 6), np.float32)
        x[:, 0] = rng.integers(40, 56, k)  # integer telemetry, occasional spike
        x[rng.random(k) < 0.01, 0] = 900.0
        x[:, 1] = rng.normal(50, 10, k)  # continuous, occasional negative spike
        x[rng.random(k) < 0.01, 1] = -1e6
        x[:, 2] = 7.0 if i < 20 else 8.0 + (i % 3)  # constant that changes
        x[:, 3] = rng.choice(np.array([1e-30, 2e-30, 3e-30], np.float32), k)
        x[rng.random(k) < 0.005, 3] = 1e30
        x[:, 4] = rng.integers(-3, 3, k) if i % 7 else np.nan  # all-NaN stretches
        x[:, 5] = t + np.arange(k)  # monotone: the range grows every push
        ts = np.arange(t, t + k, dtype=np.uint64)
        ring.push_many(x, ts)
        m.push(x)
        for rr, mm, wd in ((r16, m16, 16), (r13, m13, 13)):
            y = _rows(rng, k, wd, t)
            rr.push_many(y, ts)
            mm.push(y)
        t += k
        stream = torch.cuda.current_stream().cuda_stream
        lw.refresh(out.data_ptr(), stream)
        lwg.refresh(outg.data_ptr(), stream)
        lwo.refresh(outo.data_ptr(), stream)
        lwp.refresh(outp.data_ptr(), stream)
        lwr.refresh(outr.data_ptr(), stream)
        lwu.refresh(outu.data_ptr(), stream)
        torch.cuda.synchronize()
        _check(out, [m, m16, m13], W)
        assert torch.equal(out.nan_to_num(-7.0), outg.nan_to_num(-7.0))
        # every variant - prefetch modes, shared LDS, no compaction, brackets or the radix
        # chain alone, pass B fused into scan B or not - gives the same bits: the mean's
        # fp32 groups are fixed rows
        for o in (outo, outp, outr, outu):
            assert torch.equal(out.nan_to_num(-7.0), o.nan_to_num(-7.0))
    # brackets resolved some refreshes here and missed others (jumps, spikes, NaN stretches)
    st = lw.bracket_stats()
    assert len(st) == 35 and sum(x[1] for x in st) > 0 and any(x[1] < x[0] for x in st), st
    assert lw.stats()["fused_refreshes"] > 0 and lwu.stats()["fused_refreshes"] == 0
    assert lw.bracket_stats() == lwu.bracket_stats()  # the same hits, refresh for refresh
    assert lwr.bracket_stats() and all(x[0] == 0 for x in lwr.bracket_stats())


def test_node_refresh_one_rank_matches_local(native, cuda):
    """``refresh_node`` without a communicator (a one-rank node) runs the node-mode
    kernels - the prediction record, the combine in pass 0, the per-rank partial
    reduction read by scan 0 - and must give the local refresh's bits (last = NaN)."""
    import torch

    nat = native
    nat.set_pinned_host_rings(True)
    W, cap = 1 << 16, 1 << 14
    ra, rb = nat.SeriesRing(8, cap), nat.SeriesRing(4, cap)
    lw, lwn = nat.LongWindowSet(W, 0), nat.LongWindowSet(W, 0)
    for s in (lw, lwn):
        s.add_ring(ra)
        s.add_ring(rb)
    ma, mb = _Mirror(8), _Mirror(4)
    out, outn = torch.empty((12, 8), device=cuda), torch.empty((12, 8), device=cuda)
    rng = np.random.default_rng(21)
    t = 0
    steps = [cap, cap, cap, cap, cap, 100, 0, 3, 256, 300, 1] + [100] * 12
    for k in steps:
        xa, xb = _rows(rng, k, 8, t), _rows(rng, k, 4, -t)
        ra.push_many(xa, np.arange(t, t + k, dtype=np.uint64))
        rb.push_many(xb, np.arange(t, t + k, dtype=np.uint64))
        ma.push(xa)
        mb.push(xb)
        t += k
        stream = torch.cuda.current_stream().cuda_stream
        lw.refresh(out.data_ptr(), stream)
        lwn.refresh_node(outn.data_ptr(), stream, 50.0, 90.0, 99.0, None, False)
        torch.cuda.synchronize()
        keep = [0, 1, 2, 3, 4, 5, 7]
        assert torch.equal(out[:, keep].nan_to_num(-7.0), outn[:, keep].nan_to_num(-7.0))
        assert torch.isnan(outn[:, 6]).all()
        _check(out, [ma, mb], W)
    st = lwn.stats()
    assert st["node_refreshes"] == len(steps) and st["rows_lost"] == 0
    # node bracket mode: after the sizing refreshes, the steady 100-row pushes resolve every
    # series from the node's brackets - ties and signed zeros too (counted on exact
    # bounds) - except the monotone column of each ring (7, 11): a ramp's bracket samples
    # are consecutive rows, so one chunk's slab overflows and the radix chain resolves it
    hits = [x[1] for x in lwn.bracket_stats(1)]
    assert all(h >= 12 for s, h in enumerate(hits) if s not in (7, 11)), hits
    assert all(x[1] >= 12 for s, x in enumerate(lw.bracket_stats(0)) if s not in (7, 11)), lw.bracket_stats(0)


def test_node_long_window_one_rank_communicator():
    """The node long-window check with a one-rank RCCL communicator (the collectives run,
    timed by HIP events) at W = 2^16."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    res = subprocess.run([sys.executable, "tools/node_long_window_check.py", "--window", "65536", "--capacity",
                          "16384"], cwd=root, capture_output=True, text=True, timeout=240, env=env)
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert res.returncode == 0 and lines, (res.stdout[-3000:], res.stderr[-3000:])
    d = json.loads(lines[-1])
    assert d["ok"] and d["world"] == 1 and d["node_refreshes"] >= 8, d
    us = d["collective_us_p50"]
    assert us["bracket_records_allgather"] > 0 and us["pass3_hist_allreduce"] > 0, d
    # the steady refreshes resolve every series but the monotone ones (the last column of
    # each ring) from the node's brackets
    hits = d["node_bracket_hits"]
    assert all(h >= 12 for s, h in enumerate(hits) if s not in (7, 11)), d


@pytest.mark.parametrize("shape", ["continuous", "telemetry"])
def test_long_window_brackets_hold_in_steady_state(native, cuda, shape):
    """A filled 2^20 window that gains a few rows per refresh: continuous data - after the
    first refreshes (radix chain, then brackets sized to ~2048 samples) - is resolved by
    pass B + scan B (a select among the kept keys) with the radix chain's exact bits;
    integer telemetry stays on the one-pass radix chain."""
    import torch

    nat = native
    nat.set_pinned_host_rings(True)
    W, cap = 1 << 20, 1 << 18
    ra, rb = nat.SeriesRing(8, cap), nat.SeriesRing(4, cap)
    lw, lwr = nat.LongWindowSet(W, 0), nat.LongWindowSet(W, 0)
    lwr.brackets = False
    for s in (lw, lwr):
        s.add_ring(ra)
        s.add_ring(rb)
    ma, mb = _Mirror(8), _Mirror(4)
    out, outr = torch.empty((12, 8), device=cuda), torch.empty((12, 8), device=cuda)
    rng = np.random.default_rng(5)

    def rows(k, wd, mu):
        if shape == "telemetry":
            return rng.integers(mu - 8, mu + 8, (k, wd)).astype(np.float32)
        return rng.normal(mu, mu / 5, (k, wd)).astype(np.float32)

    t = 0
    steps = [cap] * (W // cap) + [1, 3, 0, 100, 1, 256, 7, 1, 1, 50, 1, 1]
    for k in steps:
        xa, xb = rows(k, 8, 50), rows(k, 4, 700)
        ts = np.arange(t, t + k, dtype=np.uint64)
        ra.push_many(xa, ts)
        rb.push_many(xb, ts)
        ma.push(xa)
        mb.push(xb)
        t += k
        stream = torch.cuda.current_stream().cuda_stream
        lw.refresh(out.data_ptr(), stream)
        lwr.refresh(outr.data_ptr(), stream)
        torch.cuda.synchronize()
        assert torch.equal(out.nan_to_num(-7.0), outr.nan_to_num(-7.0))
    _check(out, [ma, mb], W)
    st = lw.bracket_stats()
    # after a few refreshes sizing the brackets, every series resolved by its brackets -
    # integer telemetry too (incremental mode: a one-key bracket on the percentile's value
    # holds while its ties hold the rank)
    assert all(x[2] == 1 for x in st), st
    assert all(x[1] >= 8 for x in st), st


@pytest.mark.parametrize("shape", ["mixed", "telemetry"])
def test_incremental_brackets_stream_only_changed_chunks(native, cuda, shape):
    """Incremental bracket mode at W = 2^20 x 12 series, 100 new rows per refresh (the
    service's regime): bit-exact against bracket mode re-streaming every chunk and against
    the radix chain alone on every refresh; in the steady state pass B streams only the
    1-2 chunks per segment the new rows landed in, and the radix chain does not run."""
    import torch

    nat = native
    nat.set_pinned_host_rings(True)
    W, cap = 1 << 20, 1 << 18
    ra, rb = nat.SeriesRing(8, cap), nat.SeriesRing(4, cap)
    lw, lwf, lwr, lwu = (nat.LongWindowSet(W, 0) for _ in range(4))
    lwf.incremental = False
    lwr.brackets = False
    lwu.fused_passb = False  # incremental, pass B always its own kernel
    sets = (lw, lwf, lwr, lwu)
    for s in sets:
        s.add_ring(ra)
        s.add_ring(rb)
    ma, mb = _Mirror(8), _Mirror(4)
    outs = [torch.empty((12, 8), device=cuda) for _ in range(4)]
    rng = np.random.default_rng(17)

    def rows(k, wd, mu):
        if shape == "telemetry":
            return rng.integers(mu - 8, mu + 8, (k, wd)).astype(np.float32)
        x = rng.normal(0.0, mu / 5, (k, wd)).astype(np.float32)  # mixed sign
        x[rng.random((k, wd)) < 0.001] = np.nan  # failed reads
        return x

    t = 0
    fill = [cap] * (W // cap) + [5000]
    steps = fill + [100] * 40
    chunks_at = None
    for i, k in enumerate(steps):
        xa, xb = rows(k, 8, 50), rows(k, 4, 700)
        ts = np.arange(t, t + k, dtype=np.uint64)
        ra.push_many(xa, ts)
        rb.push_many(xb, ts)
        ma.push(xa)
        mb.push(xb)
        t += k
        stream = torch.cuda.current_stream().cuda_stream
        for s, o in zip(sets, outs):
            s.refresh(o.data_ptr(), stream)
        torch.cuda.synchronize()
        for o in outs[1:]:
            assert torch.equal(outs[0].nan_to_num(-7.0), o.nan_to_num(-7.0)), i
        if i == len(fill) + 9:
            chunks_at = (lw.stats()["passb_chunks"], lw.stats()["chain_refreshes"],
                         lw.stats()["single_kernel_refreshes"])
    _check(outs[0], [ma, mb], W)
    st = lw.stats()
    segs = 2  # the 8-series ring and the 4-series ring: one segment each
    per_refresh = (st["passb_chunks"] - chunks_at[0]) / 30
    assert per_refresh <= 2.5 * segs, (per_refresh, st)  # 100 rows land in 1-2 chunks per segment
    assert st["chain_refreshes"] - chunks_at[1] <= 3, st  # (a bracket re-centres now and then)
    assert all(x[2] == 1 for x in lw.bracket_stats()), lw.bracket_stats()
    # the steady state: scan B streams the changed chunks itself (one kernel per refresh)
    assert st["single_kernel_refreshes"] - chunks_at[2] >= 25, st
    assert lwu.stats()["fused_refreshes"] == 0 and lw.bracket_stats() == lwu.bracket_stats()
