"""locate_phases.py — time the phases of the C4 locate path on the GPU box:
ranges (search + scan + total readback), walk (expand + walk + error check),
each synchronised, 5 repetitions, and print one JSON line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from __graft_entry__ import _load_pkg  # noqa: E402


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 3_999_999_999
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 12_500_000
    m = 20
    pkg = _load_pkg()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    N = L + 1
    text = torch.empty(N + 16, dtype=torch.uint8, device=dev)
    pkg.synth_text_device("dna", 42, L, text.data_ptr(), st)
    torch.cuda.synchronize()
    idx = pkg.FMIndex.build_from_device_text(text.data_ptr(), N, pkg.BuildParams(), device=0)
    pats = torch.empty(B * m, dtype=torch.uint8, device=dev)
    offs = torch.empty(B + 1, dtype=torch.int64, device=dev)
    pkg.synth_patterns_device(text.data_ptr(), N, m, 0, B, 4242, pats.data_ptr(), offs.data_ptr(), st)
    d_sp = torch.empty(B, dtype=torch.int64, device=dev)
    d_oo = torch.empty(B + 1, dtype=torch.int64, device=dev)
    d_pos = None
    res = {"ranges_ms": [], "walk_ms": [], "walk_async_ms": []}
    for it in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tot = idx.locate_ranges_device(pats.data_ptr(), offs.data_ptr(), B, 100000,
                                       d_sp.data_ptr(), d_oo.data_ptr(), st)
        t1 = time.perf_counter()
        if d_pos is None:
            d_pos = torch.empty(tot, dtype=torch.int64, device=dev)
        idx.locate_walk_device(d_sp.data_ptr(), d_oo.data_ptr(), B, tot, d_pos.data_ptr(), st)
        t2 = time.perf_counter()
        idx.locate_walk_device(d_sp.data_ptr(), d_oo.data_ptr(), B, tot, d_pos.data_ptr(), st,
                               sync=False)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        res["ranges_ms"].append((t1 - t0) * 1e3)
        res["walk_ms"].append((t2 - t1) * 1e3)
        res["walk_async_ms"].append((t3 - t2) * 1e3)
    res["positions"] = tot
    print(json.dumps(res))


if __name__ == "__main__":
    main()
