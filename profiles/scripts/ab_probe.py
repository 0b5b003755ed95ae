#!/usr/bin/env python3
"""ab_probe.py --hook NAME=VAL [...] — the headline count (C4, Q_text 20-mers, 12.5 M) and
optional legs with and without engine hooks (read per call), alternated in one process so
box-to-box spread cancels: rounds x (A, B) kernel times from HIP events.  One JSON line.
--op locate times the one-call locate (cs_fm_locate_device, limit 100000) instead;
--hook-a NAME=VAL sets hooks for variant A (default: none)."""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hook", action="append", default=[], help="NAME=VAL for variant B (repeatable)")
    ap.add_argument("--hook-a", action="append", default=[], help="NAME=VAL for variant A (repeatable)")
    ap.add_argument("--op", default="count", choices=("count", "locate"))
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--b2b", action="store_true",
                    help="time the reps back to back between two events (as bench.py's steps)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--m", default="20")
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
    B = 12_500_000
    hooks = {"A": dict(h.split("=", 1) for h in a.hook_a), "B": dict(h.split("=", 1) for h in a.hook)}
    out = {"op": a.op, "hooks_A": hooks["A"], "hooks_B": hooks["B"], "m": {}}
    for m in [int(x) for x in a.m.split(",")]:
        W = bench.Workload(pkg, text, N, m, 0, B, "dna", "text", dev, sh)
        o = torch.empty(B + 1, dtype=torch.int64, device=dev)
        cap = 2 * B
        pos = torch.empty(cap if a.op == "locate" else 1, dtype=torch.int64, device=dev)

        def call():
            if a.op == "count":
                idx.count_batch_device(W.pats.data_ptr(), W.offs.data_ptr(), B, o.data_ptr(), sh)
            else:
                _, ok = idx.locate_device(W.pats.data_ptr(), W.offs.data_ptr(), B, 100000, o.data_ptr(),
                                          pos.data_ptr(), cap, sh)
                if not ok:
                    raise SystemExit("position capacity short")
        res = {"A": [], "B": []}
        ref = None
        for r in range(a.rounds):
            for var in ("A", "B"):
                saved = {k: os.environ.get(k) for k in list(hooks["A"]) + list(hooks["B"])}
                os.environ.update(hooks[var])
                try:
                    call()
                    torch.cuda.synchronize()
                    ms = []
                    if a.b2b:
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(st)
                        for _ in range(a.reps):
                            call()
                        e1.record(st)
                        torch.cuda.synchronize()
                        ms.append(e0.elapsed_time(e1) / a.reps)
                    for _ in range(0 if a.b2b else a.reps):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(st)
                        call()
                        e1.record(st)
                        torch.cuda.synchronize()
                        ms.append(e0.elapsed_time(e1))
                    res[var].append(statistics.mean(ms))
                    if ref is None:
                        ref = o.clone()
                    elif not torch.equal(ref, o):
                        raise SystemExit("counts differ between variants")
                finally:
                    for k, v in saved.items():
                        if v is None:
                            os.environ.pop(k, None)
                        else:
                            os.environ[k] = v
        out["m"][str(m)] = {"A_ms": res["A"], "B_ms": res["B"], "A_median": statistics.median(res["A"]),
                            "B_median": statistics.median(res["B"])}
        print("[ab] m=%d A %.4f B %.4f" % (m, statistics.median(res["A"]), statistics.median(res["B"])),
              file=sys.stderr, flush=True)
        del W, o
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
