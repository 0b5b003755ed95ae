"""The caller's workspace (cs_fm_workspace_bytes, cs_fm_count_device_ws, cs_fm_locate_device_ws;
include/cs_fmindex.h) — the path the headline count and the one-call locate bench legs run.

One workspace serves a sequence of calls: counts and one-call locates of
different batch sizes on the same memory, batches that list long patterns and general
searches for the list kernels (repetitive DNA, symbols off the table, 32..160-mers) and
batches that list nothing, a workspace that was never zero-filled (0xFF bytes: the staged
kernel claims the list kernels' retire word itself), and an undersized workspace (the call
allocates its own).  Every result is checked against the oracle (oracle/fm_oracle.c through
oracle.py), count for count and position for position."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import load_pkg

pytestmark = pytest.mark.gpu


def _dev(a, dtype):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dtype).cuda()


def _batch(text, rng, n, kind):
    """n patterns of `kind`: 'q20' text 20-mers (the one-read path, nothing listed), 'mixed'
    (20-mers, 1..31-mers, 32..160-mers, mutated copies, symbols off the table)."""
    t = np.frombuffer(text, np.uint8)
    pats = []
    for _ in range(n):
        if kind == "q20":
            m = 20
        else:
            r = rng.random()
            m = 20 if r < 0.5 else int(rng.integers(1, 32)) if r < 0.75 else int(rng.integers(32, 161))
        i = int(rng.integers(0, len(t) - m))
        p = bytearray(t[i:i + m].tobytes())
        if kind == "mixed" and rng.random() < 0.2:
            p[int(rng.integers(0, m))] = b"ACGTN"[int(rng.integers(0, 5))]
        if kind == "mixed" and rng.random() < 0.02:
            p = b""
        pats.append(bytes(p))
    return O.pack_patterns(pats)


class _Run:
    def __init__(self, pkg, text):
        self.g = pkg.FMIndex.build_from_text(text)
        self.o = O.Index(text)
        self.st = torch.cuda.current_stream().cuda_stream

    def count(self, buf, offs, ws, wsb):
        npat = len(offs) - 1
        d_p, d_o = _dev(buf, torch.uint8), _dev(offs.astype(np.int64), torch.int64)
        d_c = torch.full((npat,), -1, dtype=torch.int64, device="cuda")
        self.g.count_device_ws(d_p.data_ptr(), d_o.data_ptr(), npat, d_c.data_ptr(), ws, wsb, stream=self.st)
        torch.cuda.synchronize()
        want = self.o.count_batch(buf=buf, offs=offs, nthreads=8)
        return np.array_equal(d_c.cpu().numpy().astype(np.uint64), want)

    def locate(self, buf, offs, ws, wsb, limit=40):
        npat = len(offs) - 1
        woffs, wpos = self.o.locate_batch(buf=buf, offs=offs, limit=limit, nthreads=8)
        d_p, d_o = _dev(buf, torch.uint8), _dev(offs.astype(np.int64), torch.int64)
        d_oo = torch.full((npat + 1,), -1, dtype=torch.int64, device="cuda")
        d_pos = torch.full((max(int(woffs[-1]), 1),), -1, dtype=torch.int64, device="cuda")
        tot, ok = self.g.locate_device_ws(d_p.data_ptr(), d_o.data_ptr(), npat, limit, d_oo.data_ptr(),
                                          d_pos.data_ptr(), d_pos.numel(), ws, wsb, stream=self.st)
        torch.cuda.synchronize()
        return (ok and tot == woffs[-1] and np.array_equal(d_oo.cpu().numpy().astype(np.uint64), woffs)
                and np.array_equal(d_pos[:tot].cpu().numpy().astype(np.uint64), wpos))


@pytest.mark.parametrize("fill", [0x00, 0xFF])
@pytest.mark.parametrize("text_kind", ["dna", "rdna"])
def test_workspace_sequence(fill, text_kind):
    pkg = load_pkg()
    text = (O.gen_dna(21, 300_000) if text_kind == "dna" else O.gen_rdna(21, 300_000)).tobytes()
    r = _Run(pkg, text)
    rng = np.random.default_rng(7 if text_kind == "dna" else 8)
    big = 20_000
    wsb = r.g.workspace_bytes(big)
    ws_t = torch.full((wsb,), fill, dtype=torch.uint8, device="cuda")
    ws = ws_t.data_ptr()
    seq = [("count", "mixed", big), ("locate", "mixed", 15_000), ("count", "q20", 7_000),
           ("count", "mixed", 3_001), ("locate", "q20", big), ("count", "mixed", big),
           ("locate", "mixed", 1), ("count", "q20", 1)]
    bad = []
    for step, (op, kind, n) in enumerate(seq):
        buf, offs = _batch(text, rng, n, kind)
        ok = r.count(buf, offs, ws, wsb) if op == "count" else r.locate(buf, offs, ws, wsb)
        if not ok:
            bad.append((step, op, kind, n))
    assert not bad, bad
    # the calls leave the list counters zero (the list kernel's last block re-zeroes them)
    hdr = ws_t[:17 * 256].view(torch.int32).cpu().numpy()
    assert not hdr[::64].any(), hdr[::64]


def test_workspace_undersized_allocates():
    """work_bytes below cs_fm_workspace_bytes(npat): the call allocates its own lists."""
    pkg = load_pkg()
    text = O.gen_rdna(22, 200_000).tobytes()
    r = _Run(pkg, text)
    rng = np.random.default_rng(3)
    buf, offs = _batch(text, rng, 9_000, "mixed")
    small = r.g.workspace_bytes(100)
    ws_t = torch.full((small,), 0xFF, dtype=torch.uint8, device="cuda")
    assert r.count(buf, offs, ws_t.data_ptr(), small)
    assert r.locate(buf, offs, ws_t.data_ptr(), small)
    assert r.count(buf, offs, 0, 0)  # no workspace at all
