"""Bracket mode of the long-window statistics: the host model of ``lw_pass_brk`` +
``lw_scan_brk`` (csrc/long_window.hip "Bracket mode").

A window of W samples per series changes by the few rows that entered and left since the
previous refresh, so each percentile moves by a few ranks. The previous refresh's
percentile keys, widened by an adaptive half-width, bracket the new ones. One streaming
pass counts, per percentile q, the samples below the bracket (``lt``) and inside it
(``inn``) and keeps the keys inside; when both sorted positions of every percentile fall
inside their brackets (``lt <= pos < lt + inn``), the percentiles are order statistics of
the kept keys. Otherwise the exact radix chain resolves the series in the same refresh -
here ``np.partition``, which gives the same keys.

The half-width adapts so a bracket holds about ``target`` samples (2048, or 1/16 of a
small window). Samples ON a bound are counted, never kept (``bracket_counts``): ranks on
the lower bound are lo, past the kept keys hi. So a bracket whose bounds are tied values
- a percentile of integer telemetry, or one between two readings - holds its ranks with
no keys at all, however many samples tie. A bracket enters that exact-key form when its
value half-width gets narrower than the keys' spacing, when it overflows its kept-key cap
(read as ties), or when every kept key is the percentile's own; an exact bracket that
misses because the percentile moved to a neighbouring tied value joins the old and new
keys (a median flipping between two readings), except after an overflow. Without
incremental mode brackets are only wanted where the radix chain needs more than one
streaming pass (the varying key bits span more than pass 0's 10-bit digit).

Incremental mode (``incremental=True``, the kernels' default): a bracket that resolved a
refresh stays where it is while both positions of its percentile sit at least
``max(8, inn / 8)`` samples inside it and it holds between a quarter and twice its target -
then the per-chunk counts of the chunks no row entered stay valid and pass B streams only
the chunks that changed; only a bracket that must move is re-centred (``moves`` counts
those). Brackets are wanted for every series then (pass B costs as much as one radix pass
when it streams everything, and almost nothing when it does not).

``BracketModel.refresh(x)`` returns the same [8] statistics as ``window_stats_reference``
(min, max, mean, p50 / p90 / p99 by numpy's 'linear' rule, last, count) and whether the
brackets resolved the refresh; ``tests/test_lw_brackets.py`` checks both against numpy
over stationary, drifting, jumping and tied data.

Reference anchor: the statistics table over a window (``/root/reference/app.py:216-221``).
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

TARGET = 2048  # kBrkTarget
CAP = 8192  # kBrkCap: kept keys scan B selects among
KD0 = 10  # pass 0's widest digit
PCT = (50.0, 90.0, 99.0)


def fkey(x: np.ndarray) -> np.ndarray:
    """Order-preserving float32 -> uint32 key (csrc/long_window.hip ``fkey``)."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000).astype(np.uint64)


def kfloat(k: int) -> float:
    u = (k & 0x7FFFFFFF) if (k & 0x80000000) else (~k & 0xFFFFFFFF)
    return float(np.array([u], np.uint32).view(np.float32)[0])


def positions(nv: int, pct=PCT):
    """Sorted positions (lo, hi) and float32 weights of each percentile (lw_positions)."""
    last = nv - 1 if nv else 0
    out = []
    for p in pct:
        x = float(p) / 100.0 * float(last)
        lo = min(int(np.floor(x)), last)
        out.append((lo, lo + 1 if lo + 1 < nv else last, float(np.float32(x - lo))))
    return out


def target(nv: int, cap: int = TARGET) -> int:
    return max(64, min(cap, nv // 16))


def wanted(nv: int, minkey: int, maxkey: int, lo: int) -> bool:
    """Brackets pay when the radix chain needs more than one pass (lw_brk_wanted)."""
    d = minkey ^ maxkey
    top = d.bit_length() - 1 if d else 0
    span = top - lo + 1 if top >= lo else 1
    return bool(nv) and span > KD0


def fkey1(x: float) -> int:
    return int(fkey(np.array([x], np.float32))[0])


def est_value(minkey: int, maxkey: int, nv: int, tgt: int | None = None) -> float:
    """First half-width, in VALUE units: a quarter of the uniform density's over [min, max]
    (lw_brk_est: aims low - near a normal median the density is ~3x the uniform one)."""
    if not nv:
        return 0.0
    e = (kfloat(maxkey) - kfloat(minkey)) * (target(nv) if tgt is None else tgt) / (8.0 * nv)
    return float(np.float32(min(e, 3.0e38))) if e > 0 else 0.0


def next_bracket(delta: float, cin: int, klo: int, khi: int, est: float, had: bool, tgt: int,
                 old: tuple | None = None, join: bool = True, dsave: float = 0.0):
    """(delta, lo, hi) of the next refresh's bracket (lw_next_bracket): the half-width in
    value units, 0 = the exact keys [klo, khi]; an exact bracket that still holds ties
    joins its old keys ``old`` = (lo, hi) with the new (a percentile flipping between two
    tied readings), except after an overflow (``join`` False); one that holds few samples
    (not ties) resumes from ``dsave``, the half-width an overflow put aside, else ``est``."""
    if not had:
        d = est
    elif delta == 0.0:
        if cin >= tgt // 8:
            if join and old is not None:
                return 0.0, min(old[0], klo), max(old[1], khi)
            return 0.0, klo, khi
        d = dsave if dsave > 0.0 else est
    else:
        d = float(delta) * min(8.0, float(tgt) / float(max(cin, 1)))
    d = float(np.float32(min(d, 3.0e38)))
    if d == 0.0:
        return 0.0, klo, khi
    with np.errstate(over="ignore"):
        lo = min(klo, fkey1(np.float32(kfloat(klo)) - np.float32(d)))
        hi = max(khi, fkey1(np.float32(kfloat(khi)) + np.float32(d)))
    if klo - lo <= 1 and hi - khi <= 1:  # narrower than the keys' spacing (ties): exactly the keys
        return 0.0, klo, khi
    return d, lo, hi


@dataclass
class BracketModel:
    """One series' bracket state across refreshes."""

    lo: list = field(default_factory=lambda: [0, 0, 0])
    hi: list = field(default_factory=lambda: [0, 0, 0])
    delta: list = field(default_factory=lambda: [0.0, 0.0, 0.0])
    cin: list = field(default_factory=lambda: [0, 0, 0])
    valid: bool = False
    refreshes: int = 0
    hits: int = 0
    incremental: bool = False
    moves: int = 0  # brackets re-centred after a hit (incremental mode: their chunks restream)
    nounion: list = field(default_factory=lambda: [False, False, False])  # the last miss overflowed
    dsave: list = field(default_factory=lambda: [0.0, 0.0, 0.0])  # half-width an overflow put aside

    def refresh(self, window: np.ndarray, pct=PCT, entered: int | None = None):
        """Statistics of ``window`` (float32 samples, NaN = none) and whether the brackets
        resolved them (else the radix chain did). ``entered``: rows that entered since the
        last refresh (the incremental margin; None: unknown)."""
        x = np.asarray(window, np.float32)
        x = x[~np.isnan(x)]
        nv = int(x.size)
        out = np.full(8, np.nan)
        out[7] = nv
        if not nv:
            self.valid = False
            return out, False
        k = fkey(x)
        minkey, maxkey = int(k.min()), int(k.max())
        newest = np.float32(np.asarray(window, np.float32)[-1])
        ref = 0 if np.isnan(newest) else int(fkey(np.array([newest]))[0])  # orx's reference: the newest row
        orx = int(np.bitwise_or.reduce(k ^ np.uint64(ref)))
        lov = (orx & -orx).bit_length() - 1 if orx else 32
        pos = positions(nv, pct)
        tgt, est = target(nv), est_value(minkey, maxkey, nv)
        hit = False
        keys = [None] * 3
        ties = [False] * 3
        if self.valid:  # pass B + scan B
            self.refreshes += 1
            cnt = [bracket_counts(k, self.lo[q], self.hi[q]) for q in range(3)]
            lt = [c[0] for c in cnt]
            inn = [c[1].size + c[2] + c[3] for c in cnt]
            over = [cnt[q][1].size > CAP for q in range(3)]
            hit = all(not over[q] and lt[q] <= pos[q][0] and pos[q][1] < lt[q] + inn[q] for q in range(3))
            self.cin = inn
            if hit:
                for q in range(3):
                    keys[q], ties[q] = select_in_bracket(self.lo[q], self.hi[q], *cnt[q], pos[q])
                self.hits += 1
            else:
                for q in range(3):
                    if over[q]:  # read as ties: the next bracket is exactly the chain's keys
                        self._overflowed(q, inn[q], tgt)
        if not hit:  # the radix chain: exact keys at the sorted positions
            ks = np.sort(k)
            keys = [(int(ks[lo]), int(ks[hi])) for lo, hi, _ in pos]
        self._advance(hit, keys, ties, lt if hit else None, inn if hit else None, pos, tgt, est, entered)
        self.valid = (nv > 0) if self.incremental else wanted(nv, minkey, maxkey, lov)
        out[0], out[1] = kfloat(minkey), kfloat(maxkey)
        out[2] = np.float32(np.sum(x, dtype=np.float64) / nv)
        _percentiles(out, keys, pos)
        out[6] = float(newest)
        return out, hit

    def _overflowed(self, q, inn, tgt):
        """A miss whose bracket overflowed its kept-key cap: read as ties (the next bracket
        is exactly the chain's keys), the value half-width put aside."""
        if self.delta[q] > 0.0:
            self.dsave[q] = float(np.float32(self.delta[q] * min(8.0, tgt / max(inn, 1))))
        self.delta[q], self.nounion[q] = 0.0, True

    def _advance(self, hit, keys, ties, lt, inn, pos, tgt, est, entered):
        """The next refresh's brackets (lw_brk_resolve's t == 0 block / scan 3)."""
        had = self.valid
        for q in range(3):
            if hit and ties[q]:
                self.delta[q], self.lo[q], self.hi[q] = 0.0, keys[q][0], keys[q][0]
                self.moves += 1
                continue
            if hit and self.incremental:
                ent = inn[q] if entered is None else entered
                m = max(8, min(inn[q] // 8, 2 * ent))
                inside = pos[q][0] >= lt[q] + m and pos[q][1] + m < lt[q] + inn[q]
                # an exact-key bracket holds any number: its ties are counted, not kept
                sized = self.delta[q] == 0.0 or (inn[q] <= 2 * tgt and 4 * inn[q] >= tgt)
                if inside and sized:
                    continue  # stays put: its chunks' counts stay valid
            old = (self.lo[q], self.hi[q])
            was = self.delta[q]
            self.delta[q], self.lo[q], self.hi[q] = next_bracket(self.delta[q], self.cin[q], keys[q][0], keys[q][1],
                                                                 est, had, tgt, old, not self.nounion[q],
                                                                 self.dsave[q])
            self.nounion[q] = False
            if not (was == 0.0 and self.delta[q] == 0.0 and had and self.cin[q] >= tgt // 8):
                self.dsave[q] = 0.0  # used (or never needed): cleared, as the kernel's
            if hit and self.incremental and (self.lo[q], self.hi[q]) != old:
                self.moves += 1  # re-centred: its chunks restream (the kernels' bchg)


def bracket_counts(k: np.ndarray, lo: int, hi: int):
    """Pass B's counts of one bracket: (below, the kept keys strictly inside, on lo, on hi
    (hi != lo)) - samples on a bound are counted, never kept."""
    lo64, hi64 = np.uint64(lo), np.uint64(hi)
    lt = int(np.count_nonzero(k < lo64))
    elo = int(np.count_nonzero(k == lo64))
    ehi = int(np.count_nonzero(k == hi64)) if hi != lo else 0
    return lt, k[(k > lo64) & (k < hi64)], elo, ehi


def select_in_bracket(lo: int, hi: int, lt: int, mid: np.ndarray, elo: int, ehi: int, pos):
    """Scan B's select of one percentile inside its bracket: ranks on the lower bound are
    lo, past the kept keys hi, between them the kept keys in order. Returns ((k0, k1),
    ties): ties = every kept key is the percentile's own (-> an exact-key bracket)."""
    srt = np.sort(mid)

    def at(r):
        if r < elo:
            return lo, False
        if r < elo + srt.size:
            return int(srt[r - elo]), True
        return hi, False

    (k0, m0), (k1, m1) = at(pos[0] - lt), at(pos[1] - lt)
    ties = bool(srt.size and m0 and m1 and k0 == k1 and int(srt[0]) == k0 and int(srt[-1]) == k0)
    return (k0, k1), ties


def _percentiles(out, keys, pos):
    for q, (lo, hi, f) in enumerate(pos):
        x0, x1 = kfloat(keys[q][0]), kfloat(keys[q][1])
        out[3 + q] = np.float32(x1 - (x1 - x0) * (1.0 - f) if f >= 0.5 else x0 + (x1 - x0) * f)


NODE_TARGET = 256  # kNodeBrkTarget: node brackets hold ~256 samples of the node window
NODE_CAP = 1024  # kNodeCap: kept keys per rank and bracket in the all-gathered record
NODE_RANKS = 8  # kNodeBrkRanks: the union of the ranks' kept keys fits scan B's LDS


def node_cap_next(maxmid: int, nranks: int) -> int:
    """``lw_node_cap_next``: the next refresh's record cap (kept keys per rank and bracket
    the all-gathered records carry) from this refresh's most kept keys of any (rank, series,
    bracket) at most ``NODE_CAP`` (a bracket over it misses at any cap) - 2x headroom, a floor of 4x a rank's share of the node target, 64-key steps,
    at most ``NODE_CAP``. Every rank computes it from the same all-gathered counts."""
    c = max(2 * int(maxmid), 4 * NODE_TARGET // max(int(nranks), 1))
    return min(-(-c // 64) * 64, NODE_CAP)


@dataclass
class NodeBracketModel(BracketModel):
    """Node bracket mode (csrc/long_window.hip ``lw_node_brk_local`` + ``lw_node_brk_select``,
    host ``LongWindowSet::refresh_node``): the node's brackets - the same on every rank -
    are counted against each rank's own window; ONE all-gather of every rank's record
    (partials, below / inside counts, kept keys up to ``NODE_CAP``, rows entered) lets
    every rank select the node percentiles among the union of the kept keys. A miss (a
    position outside its bracket, a rank's bracket over its cap) falls back to the
    distributed radix chain (``node_radix_select``) in the same refresh. Incremental by
    construction (the GPU path needs it)."""

    incremental: bool = True
    chain_refreshes: int = 0
    maxmid: int = 0  # the last bracket refresh's most kept keys of one rank's bracket (node_cap_next)

    def refresh_node(self, x, allgather, allreduce_sum, pct=PCT, entered: int | None = None, cap: int = NODE_CAP):
        """Collective: ``x`` = THIS rank's window of the series (float32, NaN = none) ->
        (the node's [8] statistics over every rank's window, last = NaN; hit). ``cap``: the
        refresh's record cap (``node_cap_next`` over every series' ``maxmid``)."""
        from ..parallel.node_radix import node_radix_select

        x = np.asarray(x, np.float32)
        x = x[~np.isnan(x)]
        k = fkey(x)
        rec = {"sum": float(np.sum(x, dtype=np.float64)), "cnt": int(x.size),
               "min": int(k.min()) if x.size else 0xFFFFFFFF, "max": int(k.max()) if x.size else 0,
               "ent": None if entered is None else int(entered), "lt": [0] * 3, "in": [0] * 3, "ovf": 0,
               "keys": [None] * 3}
        rec["elo"], rec["ehi"] = [0] * 3, [0] * 3
        if self.valid:
            for q in range(3):
                lt, mid, elo, ehi = bracket_counts(k, self.lo[q], self.hi[q])
                rec["lt"][q], rec["in"][q], rec["elo"][q], rec["ehi"][q] = lt, int(mid.size), elo, ehi
                if mid.size > cap:
                    rec["ovf"] |= 1 << q
                else:
                    rec["keys"][q] = mid
        recs = allgather(rec)  # the one collective of a hit
        nv = sum(r["cnt"] for r in recs)
        out = np.full(8, np.nan)
        out[7] = nv
        if not nv:
            self.valid = False
            return out, False
        sm = 0.0
        for r in recs:  # rank order: the same mean bits on every rank
            sm += r["sum"]
        minkey, maxkey = min(r["min"] for r in recs), max(r["max"] for r in recs)
        pos = positions(nv, pct)
        tgt = target(nv, NODE_TARGET)
        est = est_value(minkey, maxkey, nv, tgt)
        ent = None if any(r["ent"] is None for r in recs) else sum(r["ent"] for r in recs)
        hit, keys, ties = False, [None] * 3, [False] * 3
        lt = [sum(r["lt"][q] for r in recs) for q in range(3)]
        mid = [sum(r["in"][q] for r in recs) for q in range(3)]
        elo = [sum(r["elo"][q] for r in recs) for q in range(3)]
        ehi = [sum(r["ehi"][q] for r in recs) for q in range(3)]
        inn = [mid[q] + elo[q] + ehi[q] for q in range(3)]
        if self.valid:
            self.refreshes += 1
            self.maxmid = max((r["in"][q] for r in recs for q in range(3) if r["in"][q] <= NODE_CAP), default=0)
            ovf = 0
            for r in recs:
                ovf |= r["ovf"]
            over = [bool((ovf >> q) & 1) or mid[q] > CAP for q in range(3)]
            hit = all(not over[q] and lt[q] <= pos[q][0] and pos[q][1] < lt[q] + inn[q] for q in range(3))
            self.cin = inn
            if hit:
                for q in range(3):
                    u = np.concatenate([r["keys"][q] for r in recs if r["keys"][q] is not None] or
                                       [np.zeros(0, np.uint64)])
                    keys[q], ties[q] = select_in_bracket(self.lo[q], self.hi[q], lt[q], u, elo[q], ehi[q], pos[q])
                self.hits += 1
            else:
                for q in range(3):
                    if over[q]:
                        self._overflowed(q, inn[q], tgt)

        if hit:
            out[0], out[1] = kfloat(minkey), kfloat(maxkey)
            out[2] = np.float32(sm / nv)
            _percentiles(out, keys, pos)
        else:  # the node radix chain (its collectives) resolves the series
            self.chain_refreshes += 1
            out = np.asarray(node_radix_select(x[None, :], pct, allgather, allreduce_sum)[0], np.float64)
            keys = self._chain_keys(x, allgather, nv, pos)
        self._advance(hit, keys, ties, lt if hit else None, inn if hit else None, pos, tgt, est, ent)
        self.valid = True
        out[6] = np.nan
        return out, hit

    @staticmethod
    def _chain_keys(x, allgather, nv, pos):
        """The exact keys at the sorted positions after a miss (the chain's scan 3 holds
        them on the GPU; here the model gathers the union - a test oracle, not the path)."""
        u = np.sort(np.concatenate(allgather(fkey(x))))
        return [(int(u[lo]), int(u[hi])) for lo, hi, _ in pos]
