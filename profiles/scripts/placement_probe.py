#!/usr/bin/env python3
"""placement_probe.py — the 0.398 -> 0.455 ms learned-lines headline (VERDICT r02 item 6:
the same kernel and PMC traffic, fast when its index is the first one a process builds, slow
after three other C4 indexes were built and freed), reproduced and separated in one process.

  1. the C4 text in HBM; a fresh 17.2-GB buffer: random 16-B reads (table_probe16, the
     count kernel's record reads without its logic) -> rate A0;
  2. the learned-lines index built first: headline count kernel time T_first, random reads
     over its own context-record table R_first;
  3. free it; build and free the bench's three other C4 indexes (default, the reference's
     wavelet matrix, walk lines) — the sequence bench.py runs before its learned legs;
  4. a fresh 17.2-GB buffer again -> A1 (translation reach / DRAM placement of memory the
     driver hands out after the frees);
  5. the learned index again: T_late, R_late.
If A1 ~ A0 but R_late < R_first, the effect is where the index's own table lands; if A1 < A0,
any memory allocated late is slower.  --arena: build every index inside one up-front
allocation instead (CS_FM_ARENA, if the engine honours it).  Prints one JSON line.
"""
import argparse
import ctypes as C
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

LIB = C.CDLL(os.path.join(ROOT, "profiles", "microbench", "libtable_probe.so"))
LIB.table_probe16.restype = C.c_float
LIB.table_probe16.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.c_int]


def probe(ptr, nbytes, reads=256_000_000):
    torch.cuda.synchronize()
    ms = float(LIB.table_probe16(ptr, nbytes, reads, 32768, 5))
    return reads / ms / 1e6  # G reads/s


def fresh_rate(nbytes, dev):
    buf = torch.empty(nbytes // 8, dtype=torch.int64, device=dev)
    buf.zero_()
    r = probe(buf.data_ptr(), nbytes)
    del buf
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return r


def headline(idx, W, B, dev, sh, reps=10):
    out = torch.empty(B, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream()
    idx.count_batch_device(W.pats.data_ptr(), W.offs.data_ptr(), B, out.data_ptr(), sh)
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        idx.count_batch_device(W.pats.data_ptr(), W.offs.data_ptr(), B, out.data_ptr(), sh)
        b.record(st)
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    del out
    return statistics.mean(ms)


def table_rate(idx):
    info = idx.info()
    meta, sizes = idx.export_meta()
    ptrs = idx.export_part_ptrs(len(sizes))
    k = max(range(len(sizes)), key=lambda i: (sizes[i] == info.prefix_bytes, sizes[i]))
    return probe(ptrs[k], sizes[k] & ~15), sizes[k]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--text-bytes", type=int, default=3_999_999_999)
    ap.add_argument("--batch", type=int, default=12_500_000)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    pkg = _load_pkg()
    sh = torch.cuda.current_stream().cuda_stream
    L = a.text_bytes
    N = L + 1
    text = torch.empty(N + 16, dtype=torch.uint8, device=dev)
    pkg.synth_text_device("dna", 42, L, text.data_ptr(), sh)
    torch.cuda.synchronize()
    W = bench.Workload(pkg, text, N, 20, 0, a.batch, "dna", "text", dev, sh)
    out = {}
    learned = {"CS_FM_ENGINE": "learned"}
    lx, _ = bench.build_index(pkg, text, N, 32, 0, learned)
    tb = lx.info().prefix_bytes
    del lx
    torch.cuda.synchronize()
    out["A0_fresh_buffer_greads_s"] = fresh_rate(tb, dev)
    lx, bs = bench.build_index(pkg, text, N, 32, 0, learned)
    out["T_first_ms"] = headline(lx, W, a.batch, dev, sh)
    out["R_first_greads_s"], out["table_bytes"] = table_rate(lx)
    del lx
    torch.cuda.synchronize()
    for env in ({}, {"CS_FM_ENGINE": "wavelet", "CS_FM_FULL_SA": "0"}, {"CS_FM_FULL_SA": "0"}):
        t0 = time.perf_counter()
        x, _ = bench.build_index(pkg, text, N, 32, 0, env)
        print("[placement] built and freed %s in %.1f s" % (env or "default", time.perf_counter() - t0),
              file=sys.stderr, flush=True)
        del x
        torch.cuda.synchronize()
    out["A1_fresh_buffer_after_frees_greads_s"] = fresh_rate(tb, dev)
    lx, _ = bench.build_index(pkg, text, N, 32, 0, learned)
    out["T_late_ms"] = headline(lx, W, a.batch, dev, sh)
    out["R_late_greads_s"], _ = table_rate(lx)
    del lx
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
