"""Serving mode (cs_fm_serve_start / FMIndex.serve): single-pattern count() answered
by a resident wave from a pinned host mailbox.  Same results as the oracle
(fm_index.cpp:79-101) and as the launch path, across every pattern length the
mailbox carries (0..124; longer ones take the launch path), symbols absent from the
text, idle exits with relaunch, concurrent callers, and shutdown by destroy."""
import threading
import time

import numpy as np
import pytest
import torch

import oracle as O
from conftest import load_pkg

pytestmark = pytest.mark.gpu


def _patterns(t, rng, n):
    pats = []
    for _ in range(n):
        m = int(rng.integers(0, 131))
        i = int(rng.integers(0, max(1, len(t) - m)))
        pats.append(t[i:i + m])
    pats += [b"", b"\xfe", t[:124], t[:125], t[:128], t[5:5 + 124] + b"\xfd", t[-3:]]
    return pats


@pytest.mark.parametrize("engine", ["auto", "wavelet", "qwm", "learned"])
@pytest.mark.parametrize("kind", ["dna", "bytes"])
def test_serve_matches_oracle(kind, engine, build_opts):
    if engine != "auto":
        build_opts(CS_FM_ENGINE=engine)
    pkg = load_pkg()
    base = (O.gen_dna(7, 20_000) if kind == "dna" else O.gen_bytes(7, 20_000)).tobytes()
    # repeats so that long patterns occur more than once
    t = base[:-1] + base[3000:3400] * 3 + base[-1:]
    g = pkg.FMIndex.build_from_text(t)
    o = O.Index(t)
    rng = np.random.default_rng(11)
    pats = _patterns(t, rng, 600)
    want = [o.count(p) for p in pats]
    g.serve(True)
    try:
        got = [g.count(p) for p in pats]
    finally:
        g.serve(False)
    assert got == want
    assert [g.count(p) for p in pats[:50]] == want[:50]  # launch path after stop


def test_serve_idle_exit_and_relaunch():
    pkg = load_pkg()
    t = O.gen_dna(8, 50_000).tobytes()
    g = pkg.FMIndex.build_from_text(t)
    o = O.Index(t)
    pats = [t[i:i + 12] for i in range(0, 40_000, 997)]
    g.serve(True, idle_us=200)
    try:
        for q, p in enumerate(pats):
            assert g.count(p) == o.count(p)
            if q % 5 == 0:
                time.sleep(0.003)  # the wave exits idle; the next request relaunches it
        g.serve(True, idle_us=200)  # already on: only the idle time changes
        assert g.count(pats[0]) == o.count(pats[0])
    finally:
        g.serve(False)
    g.serve(False)  # stopping twice is harmless


def test_serve_concurrent_callers():
    pkg = load_pkg()
    t = O.gen_dna(9, 80_000).tobytes()
    g = pkg.FMIndex.build_from_text(t)
    o = O.Index(t)
    rng = np.random.default_rng(3)
    per = [[t[i:i + m] for i, m in zip(rng.integers(0, 79_000, 150), rng.integers(1, 40, 150))]
           for _ in range(4)]
    want = [[o.count(p) for p in ps] for ps in per]
    got = [None] * 4
    g.serve(True)

    def work(k):
        got[k] = [g.count(p) for p in per[k]]

    try:
        th = [threading.Thread(target=work, args=(k,)) for k in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    finally:
        g.serve(False)
    assert got == want


def test_serve_stopped_by_destroy():
    pkg = load_pkg()
    t = O.gen_dna(10, 10_000).tobytes()
    g = pkg.FMIndex.build_from_text(t)
    g.serve(True, idle_us=10_000_000)  # would stay resident for the 10 s lifetime cap
    assert g.count(t[100:110]) == O.Index(t).count(t[100:110])
    del g  # cs_fm_destroy stops the wave
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 1.0
