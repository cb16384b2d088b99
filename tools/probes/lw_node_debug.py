"""Bracket-mode diagnosis on one GPU: the stream of tests/test_gpu_long_window.py's
node test through a local LongWindowSet (mode 0) and a one-rank node one (mode 1, no
communicator), next to the numpy models (rocmdash.runtime.lw_brackets). Per refresh, which
series each resolved from its brackets, and for a series where the GPU and the model
disagree, both bracket records. One JSON line per refresh.

    python tools/probes/lw_node_debug.py [--steady 12]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steady", type=int, default=12)
    ap.add_argument("--window", type=int, default=1 << 16)
    args = ap.parse_args()
    import numpy as np
    import torch

    from rocmdash.runtime import native
    from rocmdash.runtime.lw_brackets import BracketModel, NodeBracketModel, kfloat
    from test_gpu_long_window import _rows

    nat = native.load()
    nat.set_pinned_host_rings(True)
    W, cap = args.window, 1 << 14
    ra, rb = nat.SeriesRing(8, cap), nat.SeriesRing(4, cap)
    lw, lwn = nat.LongWindowSet(W, 0), nat.LongWindowSet(W, 0)
    for s in (lw, lwn):
        s.add_ring(ra)
        s.add_ring(rb)
    out, outn = torch.empty((12, 8), device="cuda"), torch.empty((12, 8), device="cuda")
    rng = np.random.default_rng(21)
    A, B = np.zeros((0, 8), np.float32), np.zeros((0, 4), np.float32)
    nm = [NodeBracketModel() for _ in range(12)]
    lm = [BracketModel(incremental=True) for _ in range(12)]
    t = 0
    steps = [cap] * (W // cap + 1) + [100, 0, 3, 256, 300, 1] + [100] * args.steady
    bad = 0
    for i, k in enumerate(steps):
        xa, xb = _rows(rng, k, 8, t), _rows(rng, k, 4, -t)
        ra.push_many(xa, np.arange(t, t + k, dtype=np.uint64))
        rb.push_many(xb, np.arange(t, t + k, dtype=np.uint64))
        A, B = np.concatenate([A, xa])[-W:], np.concatenate([B, xb])[-W:]
        t += k
        X = np.concatenate([A, B], axis=1)
        stream = torch.cuda.current_stream().cuda_stream
        st0, stn0 = lw.stats(), lwn.stats()
        lw.refresh(out.data_ptr(), stream)
        lwn.refresh_node(outn.data_ptr(), stream, 50.0, 90.0, 99.0, None, False)
        torch.cuda.synchronize()
        g0, g1 = lw.bracket_state(0), lwn.bracket_state(1)
        mh_l, mh_n = [], []
        for s in range(12):
            mh_n.append(nm[s].refresh_node(X[:, s], lambda o: [o], lambda a: a, entered=k)[1])
            mh_l.append(lm[s].refresh(X[:, s], entered=k)[1])
        st1, stn1 = lw.stats(), lwn.stats()
        rec = {"i": i, "rows": k,
               "local_gpu": "".join("1" if g0[s]["hit"] and st1["bracket_refreshes"] > st0["bracket_refreshes"] else "."
                                    for s in range(12)) if g0 else None,
               "local_model": "".join("1" if h else "." for h in mh_l),
               "node_gpu": "".join("1" if g1[s]["hit"] and stn1["bracket_refreshes"] > stn0["bracket_refreshes"] else "."
                                   for s in range(12)) if g1 else None,
               "node_model": "".join("1" if h else "." for h in mh_n),
               "chain_local": st1["chain_refreshes"] - st0["chain_refreshes"],
               "chain_node": stn1["chain_refreshes"] - stn0["chain_refreshes"],
               "passb_chunks_node": stn1["passb_chunks"] - stn0["passb_chunks"]}
        diff = []
        if g1 and i >= len(steps) - args.steady:
            for s in range(12):
                if bool(g1[s]["hit"]) != mh_n[s]:
                    m = nm[s]
                    diff.append({"s": s, "gpu": {"lo": [kfloat(x) for x in g1[s]["lo"]],
                                                 "hi": [kfloat(x) for x in g1[s]["hi"]],
                                                 "delta": g1[s]["delta"], "cin": g1[s]["cin"],
                                                 "valid": g1[s]["valid"], "nounion": g1[s]["nounion"]},
                                 "model": {"lo": [kfloat(x) for x in m.lo], "hi": [kfloat(x) for x in m.hi],
                                           "delta": m.delta, "cin": m.cin}})
        if diff:
            rec["diff"] = diff[:4]
            bad += 1
        print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
