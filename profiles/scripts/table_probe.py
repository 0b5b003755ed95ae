#!/usr/bin/env python3
"""table_probe.py [bench config args] — random 16-B reads from an index's own prefix table
vs. from a freshly allocated buffer of the same size, on the same GPU in one process.

Question: is the C3 count kernel slow because its 69-GB table sits
in memory the build fragmented (address-translation misses), or because of the kernel?
Both probes are the same HIP kernel (gather_bench's independent random 16-B reads,
profiles/microbench/table_probe.hip), so only the placement of the table differs.  Prints one JSON line.
  python profiles/scripts/table_probe.py --kind bytes --text-bytes 999999999   (C3)
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from __graft_entry__ import _load_pkg  # noqa: E402


_LIB = None


def probe(ptr, nbytes, reads, grid=32768, reps=5):
    """mean ms of `reads` independent random 16-B reads over [ptr, ptr + nbytes)
    (profiles/microbench/table_probe.hip: gather_bench's k_indep<16>)."""
    global _LIB
    import ctypes as C
    if _LIB is None:
        _LIB = C.CDLL(os.path.join(ROOT, "profiles", "microbench", "libtable_probe.so"))
        _LIB.table_probe16.restype = C.c_float
        _LIB.table_probe16.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.c_int]
        _LIB.table_probe_shape.restype = C.c_float
        _LIB.table_probe_shape.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.c_int, C.c_int]
    torch.cuda.synchronize()
    return float(_LIB.table_probe16(ptr, nbytes, reads, grid, reps))


def probe_shape(ptr, nbytes, npat, u, grid, reps=5):
    """mean ms of the count kernels' shape over npat patterns: U per lane, one-shot lanes
    (grid 0) or a fixed grid of looping lanes (table_probe.hip k_shape)."""
    probe(ptr, 1 << 20, 1 << 20)  # loads the library
    torch.cuda.synchronize()
    return float(_LIB.table_probe_shape(ptr, nbytes, npat, u, grid, reps))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="bytes")
    ap.add_argument("--text-bytes", type=int, default=999_999_999)
    ap.add_argument("--reads", type=int, default=256_000_000)
    ap.add_argument("--npat", type=int, default=10_000_000, help="patterns of the shape probes")
    a = ap.parse_args()
    pkg = _load_pkg()
    dev = torch.device("cuda", 0)
    N = a.text_bytes + 1
    text = torch.empty(N + 16, dtype=torch.uint8, device=dev)
    pkg.synth_text_device(a.kind, 42, a.text_bytes, text.data_ptr(), 0)
    idx = pkg.FMIndex.build_from_device_text(text.data_ptr(), N, pkg.BuildParams(ssa_stride=32), device=0)
    torch.cuda.synchronize()
    del text
    info = idx.info()
    meta, sizes = idx.export_meta()
    ptrs = idx.export_part_ptrs(len(sizes))
    # the prefix table is the part of prefix_bytes
    k = max(range(len(sizes)), key=lambda i: (sizes[i] == info.prefix_bytes, sizes[i]))
    nb = sizes[k] & ~15
    t_index = probe(ptrs[k], nb, a.reads)
    fresh = torch.empty(nb // 8, dtype=torch.int64, device=dev)
    fresh.random_()
    t_fresh = probe(fresh.data_ptr(), nb, a.reads)
    shapes = {}
    for u in (1, 2, 4):
        for grid in (0, 2048, 8192):
            ms = probe_shape(ptrs[k], nb, a.npat, u, grid)
            shapes["u%d_grid%d" % (u, grid)] = {"ms": ms, "greads_s": a.npat / ms / 1e6}
    print(json.dumps({"shapes": shapes, "npat": a.npat, "table_bytes": nb, "reads": a.reads, "prefix_k": info.prefix_k,
                      "record_bytes": info.record_bytes,
                      "index_table_ms": t_index, "index_table_greads_s": a.reads / t_index / 1e6,
                      "fresh_buffer_ms": t_fresh, "fresh_buffer_greads_s": a.reads / t_fresh / 1e6}))


if __name__ == "__main__":
    main()
