"""The long-window passes' chunking (csrc/long_window.hip ``long_window_chunk_plan``): per
ring, rows per workgroup and workgroups per 8-series segment. Planned chunks give every
workgroup about the same bytes (the passes are latency-bound per wave, so the slowest
workgroup sets a pass's time) in whole rounds of the chip's workgroup slots, within the
16-bit LDS bins; a caller's chunk_rows is used as given for every ring."""

import pytest

LAYOUTS = [[8, 4], [8], [4], [12], [4, 4, 4], [16, 16, 16, 16], [1], [16, 3]]
WINDOWS = [1 << 15, 1 << 16, 1 << 20, 1 << 22, 1 << 24, 1 << 26]
MAX_ROWS = 65280  # kLongChunkRowsMax: 16-bit LDS bins


def _segs(w):
    return (w + 7) // 8


@pytest.mark.parametrize("W", WINDOWS)
@pytest.mark.parametrize("widths", LAYOUTS)
def test_plan_covers_the_window_within_the_bins(native, W, widths):
    plan = native.long_window_chunk_plan(W, widths, 256)
    assert len(plan) == len(widths)
    for rows, n in plan:
        assert rows % 256 == 0 and 256 <= rows <= MAX_ROWS
        assert (n - 1) * rows < W <= n * rows  # every row in exactly one chunk, no empty chunk


@pytest.mark.parametrize("W", [1 << 22, 1 << 24, 1 << 26])
@pytest.mark.parametrize("widths", LAYOUTS)
def test_plan_balances_bytes_in_whole_rounds(native, W, widths):
    cus = 256
    plan = native.long_window_chunk_plan(W, widths, cus)
    slots = 4 * cus
    wgs = sum(n * _segs(w) for (rows, n), w in zip(plan, widths))
    rounds = -(-wgs // slots)
    assert wgs <= rounds * slots and wgs > (rounds - 1) * slots + slots // 2  # a round is nearly full
    # bytes one workgroup streams: rows x the segment's series x 4 B, within 10 % over rings
    per_wg = [rows * min(w, 8) * 4 for (rows, n), w in zip(plan, widths) if w >= 4]
    if len(per_wg) > 1:
        assert max(per_wg) <= 1.1 * min(per_wg), (plan, per_wg)


def test_service_layout_at_2p24(native):
    # the service's rings (8 + 4 series): 683 x 24576 rows and 340 x 49408 rows - 1023
    # workgroups of ~770 KB, where uniform 32768-row chunks gave 512 of 1 MB + 512 of 0.5 MB
    assert native.long_window_chunk_plan(1 << 24, [8, 4], 256) == [(24576, 683), (49408, 340)]
    assert native.long_window_chunk_plan(1 << 24, [8, 4], 256, 32768) == [(32768, 512), (32768, 512)]


def test_plan_follows_the_compute_units(native):
    # a partitioned device (CPX: 32 CUs, 128 slots) gets one round of its own slots, or
    # two when one round would need more rows per workgroup than the bins hold
    assert sum(n for _, n in native.long_window_chunk_plan(1 << 20, [8, 4], 32)) <= 128
    assert 128 < sum(n for _, n in native.long_window_chunk_plan(1 << 22, [8, 4], 32)) <= 256


@pytest.mark.parametrize("window,widths,chunk", [(1 << 20, [0], 0), (1 << 20, [17], 0), (3 << 20, [8], 0),
                                                 (512, [8], 0), (1 << 20, [], 0), (1 << 20, [8] * 5, 0),
                                                 (1 << 20, [8], 300)])
def test_chunk_plan_rejects_bad_inputs(native, window, widths, chunk):
    """The exposed planner validates what it is given instead of searching forever
    (ADVICE r04): widths in [1, 16], 1-4 rings, a power-of-two window in [2^10, 2^26]."""
    with pytest.raises(ValueError):
        native.long_window_chunk_plan(window, widths, 256, chunk)


def test_plan_rounds_make_smaller_chunks(native):
    """More rounds of the chip's workgroup slots: smaller chunks (the incremental pass B
    re-streams fewer rows per changed chunk)."""
    one = native.long_window_chunk_plan(1 << 24, [8, 4], 256)
    three = native.long_window_chunk_plan(1 << 24, [8, 4], 256, 0, 3)
    # (incremental plans: every ring the smallest ring's chunk - pass B's column-split
    # workgroups stream chunk_rows rows whatever the ring's width)
    assert three == [(8192, 2048), (8192, 2048)], three
    assert all(r3 < r1 for (r3, _), (r1, _) in zip(three, one))
    with pytest.raises(ValueError):
        native.long_window_chunk_plan(1 << 24, [8, 4], 256, 0, 0)
