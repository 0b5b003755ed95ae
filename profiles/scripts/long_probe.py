#!/usr/bin/env python3
"""long_probe.py [--text-bytes N] [--batch B] [--m 64,150] [--variants ...] — the long-pattern
count forms on one index, one process (round 3).

Builds the C4 index once (default 4e9 DNA), then for each pattern length m times the count of
a Q_text batch through: the staged kernel alone (flags 0, CS_FM_LONG_ROUTE=0: k_count_ctx ->
general search; the reference for the equality check), the default path (flags 0: routed to
k_count_long after the first call) and CS_Q_LONG with each CS_FM_LONG_KERNEL value.  Kernel time from HIP events on the launch stream (mean of --reps after a
warm-up); every variant's counts must equal the default path's.  Prints one JSON line.
"""
import argparse
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (Workload, build_index)
from __graft_entry__ import _load_pkg  # noqa: E402


def timed(fn, reps, stream):
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        fn()
        b.record(stream)
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    return statistics.mean(ms), min(ms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--text-bytes", type=int, default=3_999_999_999)
    ap.add_argument("--batch", type=int, default=12_500_000)
    ap.add_argument("--m", default="33,64,150")
    ap.add_argument("--variants", default="0,2,1",
                    help="CS_FM_LONG_KERNEL values: 0 round 2's kernel, 2 k_count_long on the byte "
                         "text, 1 k_count_long on the packed text (the default)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kind", default="dna")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    pkg = _load_pkg()
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    L = args.text_bytes
    N = L + 1
    text = torch.empty(N + 16, dtype=torch.uint8, device=dev)
    pkg.synth_text_device(args.kind, 42, L, text.data_ptr(), sh)
    torch.cuda.synchronize()
    idx, bs = bench.build_index(pkg, text, N, 32, 0)
    info = idx.info()
    out = {"n": N, "batch": args.batch, "build_s": bs, "packed_text_bytes": info.packed_text_bytes,
           "lengths": {}}
    B = args.batch
    for m in [int(x) for x in args.m.split(",")]:
        W = bench.Workload(pkg, text, N, m, 0, B, args.kind, "text", dev, sh)
        ref = torch.empty(B, dtype=torch.int64, device=dev)
        o8 = torch.empty(B, dtype=torch.int64, device=dev)
        row = {}
        os.environ["CS_FM_LONG_ROUTE"] = "0"
        mean, mn = timed(lambda: idx.count_device_ex(W.pats.data_ptr(), W.offs.data_ptr(), B, ref.data_ptr(),
                                                     flags=0, stream=sh), args.reps, stream)
        os.environ.pop("CS_FM_LONG_ROUTE")
        row["staged_only"] = {"ms": mean, "ms_min": mn, "patterns_per_s": B / mean * 1e3}
        want = ref.clone()
        # the default path: the warm-up call raises the routing flag, the timed calls route
        o8.fill_(-1)
        mean, mn = timed(lambda: idx.count_device_ex(W.pats.data_ptr(), W.offs.data_ptr(), B, o8.data_ptr(),
                                                     flags=0, stream=sh), args.reps, stream)
        row["default_routed"] = {"ms": mean, "ms_min": mn, "patterns_per_s": B / mean * 1e3,
                                 "matches": bool(torch.equal(o8, want))}
        print("[long_probe] m=%d staged %.3f routed %.3f ms" % (m, row["staged_only"]["ms"], mean),
              file=sys.stderr, flush=True)
        for v in args.variants.split(","):
            # a CS_FM_LONG_KERNEL value, or KEY=VAL[+KEY=VAL] engine hooks
            env = dict(x.split("=", 1) for x in v.split("+")) if "=" in v else {"CS_FM_LONG_KERNEL": v}
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                o8.fill_(-1)
                mean, mn = timed(lambda: idx.count_device_ex(W.pats.data_ptr(), W.offs.data_ptr(), B,
                                                             o8.data_ptr(), flags=32, stream=sh),
                                 args.reps, stream)
                ok = bool(torch.equal(o8, want))
            finally:
                for k, x in saved.items():
                    if x is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = x
            row["long_" + v] = {"ms": mean, "ms_min": mn, "patterns_per_s": B / mean * 1e3,
                                "matches_default": ok}
            print("[long_probe] m=%d %s %.3f ms %s" % (m, v, mean, ok), file=sys.stderr, flush=True)
        row["found_frac"] = float((want >= 1).float().mean().item())
        out["lengths"][str(m)] = row
        del W, ref, o8, want
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
