"""p50_breakdown.py — single-pattern count() latency on C4 by pattern shape:
empty pattern (launch + result round trip only), 14-mer (prefix table only),
16/18/20-mers (table + 2/4/6 rank steps); launch path (one kernel per call) and
serving mode (FMIndex.serve: a resident wave answers from a pinned mailbox)."""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from __graft_entry__ import _load_pkg  # noqa: E402


def main():
    pkg = _load_pkg()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    L = 3_999_999_999
    N = L + 1
    text = torch.empty(N + 16, dtype=torch.uint8, device=dev)
    pkg.synth_text_device("dna", 42, L, text.data_ptr(), st)
    torch.cuda.synchronize()
    idx = pkg.FMIndex.build_from_device_text(text.data_ptr(), N, pkg.BuildParams(), device=0)
    npat = 2000
    pats = torch.empty(npat * 20, dtype=torch.uint8, device=dev)
    pkg.synth_patterns_device(text.data_ptr(), N, 20, 0, npat, 4242, pats.data_ptr(), None, st)
    torch.cuda.synchronize()
    hp = pats.cpu().numpy().reshape(npat, 20)
    res = {}
    for mode in ("launch", "serve"):
        if mode == "serve":
            idx.serve(True)
        for m in (0, 14, 16, 18, 20):
            lat = []
            for q in range(npat):
                b = hp[q, 20 - m:].tobytes()
                t0 = time.perf_counter()
                idx.count(b)
                lat.append((time.perf_counter() - t0) * 1e6)
            res["%s_m%d_p50_us" % (mode, m)] = statistics.median(lat[100:])
        if mode == "serve":
            idx.serve(False)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
