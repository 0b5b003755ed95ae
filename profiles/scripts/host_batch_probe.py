"""host_batch_probe.py — where the time of a large host batch goes (cs_fm_count_batch with
host arrays): 12.5 M Q_text 20-mers over a 100 MB DNA index, the call timed whole with
(a) the batch in one piece (CS_FM_HOST_CHUNK=10^9) and (b) in chunks whose caller pages
are page-locked piece by piece (default 2 M, and 4 M), with the counts array fresh
(untouched pages) or reused; plus the host-side offsets check alone (numpy) and a plain
pinned H2D copy of the same bytes.  Prints one JSON object."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import __graft_entry__ as G  # noqa: E402

pkg = G._load_pkg()
torch.cuda.set_device(0)
N = 100_000_000
text = torch.empty(N + 16, dtype=torch.uint8, device="cuda")
pkg.synth_text_device("dna", 42, N - 1, text.data_ptr(), 0)
g = pkg.FMIndex.build_from_device_text(text.data_ptr(), N, pkg.BuildParams(ssa_stride=32))
B, m = 12_500_000, 20
d_p = torch.empty(B * m, dtype=torch.uint8, device="cuda")
d_o = torch.empty(B + 1, dtype=torch.int64, device="cuda")
pkg.synth_patterns_device(text.data_ptr(), N, m, 0, B, 4242, d_p.data_ptr(), d_o.data_ptr(), 0)
torch.cuda.synchronize()
hp = d_p.cpu().numpy()
ho = d_o.cpu().numpy().astype(np.uint64)
lib = pkg.lib()
res = {"patterns": B, "m": m}

t0 = time.perf_counter()
ok = bool((ho[1:] >= ho[:-1]).all())
res["offsets_check_numpy_ms"] = (time.perf_counter() - t0) * 1e3


def call(out):
    t0 = time.perf_counter()
    st = lib.cs_fm_count_batch(g._h, pkg._u8(hp), pkg._u64(ho), B, pkg._u64(out), None)
    assert st == 0, lib.cs_fm_last_error()
    return (time.perf_counter() - t0) * 1e3


want = None
for chunk in ("1000000000", "2097152", "4194304", "1048576"):
    os.environ["CS_FM_HOST_CHUNK"] = chunk
    reuse = np.ones(B, np.uint64)
    call(reuse)
    t_reuse = min(call(reuse) for _ in range(3))
    t_fresh = min(call(np.zeros(B, np.uint64)) for _ in range(3))
    if want is None:
        want = reuse.copy()
    res["chunk_" + chunk] = {"ms_reused_out": t_reuse, "ms_fresh_out": t_fresh,
                             "patterns_per_s_reused": B / t_reuse * 1e3,
                             "matches": bool(np.array_equal(reuse, want))}
pin = torch.from_numpy(hp).pin_memory()
dst = torch.empty_like(d_p)
dst.copy_(pin, non_blocking=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
dst.copy_(pin, non_blocking=True)
torch.cuda.synchronize()
res["pinned_h2d_patterns_ms"] = (time.perf_counter() - t0) * 1e3
print(json.dumps(res))
