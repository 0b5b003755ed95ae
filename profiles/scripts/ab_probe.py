#!/usr/bin/env python3
"""ab_probe.py --flags-b QT_NAME[,QT_NAME] — the headline count (C4, Q_text 20-mers, 12.5 M) and
optional pattern lengths with and without tuning selectors (cs_fmindex.h CS_QT_*: per-call
flags bits, round 5 — no environment is read by a query), alternated in one process so
box-to-box spread cancels: rounds x (A, B) times from HIP events.  One JSON line.
--op locate times the one-call locate (limit 100000) instead; --flags-a sets variant A's bits
(default: none); --b2b times the reps back to back between two events (as bench.py's steps);
--ws-a / --ws-b give a variant the caller's workspace (cs_fm_*_ws) instead of the per-call
allocation."""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from __graft_entry__ import _load_pkg  # noqa: E402


def flag_bits(pkg, spec):
    b = 0
    for name in filter(None, (spec or "").split(",")):
        b |= getattr(pkg, name if name.startswith("Q") else "QT_" + name)
    return b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags-a", default="", help="tuning bits of variant A (QT_* names, comma-separated)")
    ap.add_argument("--flags-b", default="", help="tuning bits of variant B")
    ap.add_argument("--ws-a", action="store_true", help="variant A with a workspace")
    ap.add_argument("--ws-b", action="store_true", help="variant B with a workspace")
    ap.add_argument("--op", default="count", choices=("count", "locate"))
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--b2b", action="store_true")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--m", default="20")
    ap.add_argument("--batch", type=int, default=12_500_000)
    ap.add_argument("--text-kind", default="dna", help="dna or rdna")
    ap.add_argument("--text-bytes", type=int, default=3_999_999_999)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    pkg = _load_pkg()
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    N = a.text_bytes + 1
    text = torch.empty(N + 16, dtype=torch.uint8, device=dev)
    pkg.synth_text_device(a.text_kind, 42, a.text_bytes, text.data_ptr(), sh)
    torch.cuda.synchronize()
    idx, _ = bench.build_index(pkg, text, N, 32, 0)
    B = a.batch
    fl = {"A": flag_bits(pkg, a.flags_a), "B": flag_bits(pkg, a.flags_b)}
    use_ws = {"A": a.ws_a, "B": a.ws_b}
    wsb = idx.workspace_bytes(B)
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    out = {"op": a.op, "flags_A": a.flags_a, "flags_B": a.flags_b, "ws_A": a.ws_a, "ws_B": a.ws_b,
           "batch": B, "text_kind": a.text_kind, "b2b": a.b2b, "m": {}}
    for m in [int(x) for x in a.m.split(",")]:
        W = bench.Workload(pkg, text, N, m, 0, B, "dna", "text", dev, sh)
        o = torch.empty(B + 1, dtype=torch.int64, device=dev)
        cap = 2 * B
        pos = torch.empty(cap if a.op == "locate" else 1, dtype=torch.int64, device=dev)

        def call(var):
            w, wb = (ws.data_ptr(), wsb) if use_ws[var] else (0, 0)
            if a.op == "count":
                idx.count_device_ws(W.pats.data_ptr(), W.offs.data_ptr(), B, o.data_ptr(), w, wb,
                                    flags=fl[var], stream=sh)
            else:
                _, ok = idx.locate_device_ws(W.pats.data_ptr(), W.offs.data_ptr(), B, 100000, o.data_ptr(),
                                             pos.data_ptr(), cap, w, wb, sh, flags=fl[var])
                if not ok:
                    raise SystemExit("position capacity short")
        res = {"A": [], "B": []}
        ref = None
        for r in range(a.rounds):
            for var in ("A", "B"):
                call(var)
                torch.cuda.synchronize()
                ms = []
                if a.b2b:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(a.reps):
                        call(var)
                    e1.record(st)
                    torch.cuda.synchronize()
                    ms.append(e0.elapsed_time(e1) / a.reps)
                for _ in range(0 if a.b2b else a.reps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    call(var)
                    e1.record(st)
                    torch.cuda.synchronize()
                    ms.append(e0.elapsed_time(e1))
                res[var].append(statistics.median(ms))
                if ref is None:
                    ref = o.clone()
                elif not torch.equal(ref, o):
                    raise SystemExit("results differ between variants")
        out["m"][str(m)] = {"A_ms": res["A"], "B_ms": res["B"], "A_median": statistics.median(res["A"]),
                            "B_median": statistics.median(res["B"])}
        print("[ab] m=%d A %.4f B %.4f" % (m, statistics.median(res["A"]), statistics.median(res["B"])),
              file=sys.stderr, flush=True)
        del W, o
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
