#!/usr/bin/env python3
"""stream_probe.py — the headline count (C4, Q_text 20-mers, 12.5 M per call) issued back to
back on one stream against the same calls alternating over S streams (each stream its own
workspace and output), wall time of K calls between two device synchronisations; rounds
alternate the forms in one process.  Also times one 100 M call over the same generator's
batch (BASELINE configs[3]).  What it answers: how much of a call's time is the staged
kernel's head and tail (the last blocks draining while the next call's cannot start), which
independent batches on separate streams overlap.  One JSON line."""
import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from __graft_entry__ import _load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,2,3")
    ap.add_argument("--calls", type=int, default=48)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batch", type=int, default=12_500_000)
    ap.add_argument("--text-bytes", type=int, default=3_999_999_999)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    pkg = _load_pkg()
    st0 = torch.cuda.current_stream()
    N = a.text_bytes + 1
    text = torch.empty(N + 16, dtype=torch.uint8, device=dev)
    pkg.synth_text_device("dna", 42, a.text_bytes, text.data_ptr(), st0.cuda_stream)
    torch.cuda.synchronize()
    idx, _ = bench.build_index(pkg, text, N, 32, 0)
    B = a.batch
    W = bench.Workload(pkg, text, N, 20, 0, B, "dna", "text", dev, st0.cuda_stream)
    torch.cuda.synchronize()
    smax = max(int(x) for x in a.streams.split(","))
    streams = [torch.cuda.Stream() for _ in range(smax)]
    wsb = idx.workspace_bytes(B)
    ws = [torch.zeros(wsb, dtype=torch.uint8, device=dev) for _ in range(smax)]
    outs = [torch.empty(B + 1, dtype=torch.int64, device=dev) for _ in range(smax)]
    torch.cuda.synchronize()

    host_us = []

    def run(S):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.calls):
            s = i % S
            idx.count_device_ws(W.pats.data_ptr(), W.offs.data_ptr(), B, outs[s].data_ptr(), ws[s].data_ptr(), wsb,
                                stream=streams[s].cuda_stream)
        t1 = time.perf_counter()  # (the host's issue time: the device runs behind it)
        torch.cuda.synchronize()
        host_us.append((t1 - t0) * 1e6 / a.calls)
        return (time.perf_counter() - t0) * 1e3 / a.calls

    forms = [int(x) for x in a.streams.split(",")]
    for S in forms:  # warm-up
        run(S)
    res = {S: [] for S in forms}
    for _ in range(a.rounds):
        for S in forms:
            res[S].append(run(S))
    ref = outs[0].clone()
    for s in range(1, smax):
        if not torch.equal(outs[s], ref):
            raise SystemExit("stream outputs differ")
    out = {"batch": B, "calls": a.calls, "host_issue_us_per_call": statistics.median(host_us),
           "ms_per_call": {str(S): statistics.median(v) for S, v in res.items()},
           "rounds": {str(S): v for S, v in res.items()}}
    # a C2-sized batch (1 M patterns) on the same index, 1 and 2 streams: the fixed per-call
    # costs (launches, the empty list kernel, head and tail) weigh 12.5x more there
    Bs = 1_000_000
    for S in forms:
        res[S] = []
    for _ in range(a.rounds):
        for S in forms:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.calls):
                s = i % S
                idx.count_device_ws(W.pats.data_ptr(), W.offs.data_ptr(), Bs, outs[s].data_ptr(), ws[s].data_ptr(),
                                    wsb, stream=streams[s].cuda_stream)
            torch.cuda.synchronize()
            res[S].append((time.perf_counter() - t0) * 1e3 / a.calls)
    out["ms_per_call_1m"] = {str(S): statistics.median(v) for S, v in res.items()}
    # one call over the whole 100 M batch (BASELINE configs[3]), same generator
    del ws, outs
    B8 = 8 * B
    W8 = bench.Workload(pkg, text, N, 20, 0, B8, "dna", "text", dev, st0.cuda_stream)
    o8 = torch.empty(B8 + 1, dtype=torch.int64, device=dev)
    ws8b = idx.workspace_bytes(B8)
    ws8 = torch.zeros(ws8b, dtype=torch.uint8, device=dev)
    sh = st0.cuda_stream
    ms8 = []
    for r in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        idx.count_device_ws(W8.pats.data_ptr(), W8.offs.data_ptr(), B8, o8.data_ptr(), ws8.data_ptr(), ws8b, stream=sh)
        torch.cuda.synchronize()
        if r:
            ms8.append((time.perf_counter() - t0) * 1e3)
    out["ms_100m_per_12p5m"] = statistics.median(ms8) / 8
    if not torch.equal(o8[:B], ref[:B]):
        raise SystemExit("100 M batch's first 12.5 M differ")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
