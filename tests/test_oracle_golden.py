"""Pin the CPU restatement (oracle/) against the genuine reference's golden vectors.

CPU-only.  The fixtures in tests/golden/ were produced by the reference itself
(tests/golden/make_golden.py driving oracle/_ref/).  Both rank modes of the oracle
(faithful = reference cost model, fast = precomputed totals) must reproduce them
bit for bit, quirks included (cyclic BWT without terminator, duplicate '$', row
order, limit truncation, the LF-overrun exception).
"""
import numpy as np
import pytest

import oracle as O
from conftest import fm_golden_cases, golden_text, load_golden


def _check_fm_case(case, faithful):
    text = golden_text(case["text"])
    assert len(text) == case["n"]
    idx = O.Index(text, ssa_stride=case["ssa_stride"])
    for ph, cnt, loc in zip(case["patterns_hex"], case["count"], case["locate"]):
        p = bytes.fromhex(ph)
        assert idx.count(p, faithful=faithful) == cnt, (case["name"], p)
        if "error" in loc:
            with pytest.raises(RuntimeError) as ei:
                idx.locate(p, limit=case["limit"], faithful=faithful)
            if loc["error"] != "exception":
                assert str(ei.value) == loc["error"]
        else:
            assert idx.locate(p, limit=case["limit"], faithful=faithful) == loc["pos"], (case["name"], p)
    for ex in case.get("extract", []):
        assert idx.extract(ex["pos"], ex["len"]).hex() == ex["hex"]


@pytest.mark.parametrize("case", fm_golden_cases("fm_kat.json"))
@pytest.mark.parametrize("faithful", [True, False])
def test_fm_kat(case, faithful):
    _check_fm_case(case, faithful)


@pytest.mark.parametrize("case", fm_golden_cases("fm_100k.json", "fm_1m.json"))
def test_fm_large_fast(case):
    _check_fm_case(case, faithful=False)


def test_fm_100k_faithful_sample():
    """Faithful mode (with the O(n) count_ones scans) on a sample of the 1e5 case."""
    case = load_golden("fm_100k.json")["cases"][0]
    text = golden_text(case["text"])
    idx = O.Index(text, ssa_stride=case["ssa_stride"])
    for k in range(0, len(case["patterns_hex"]), 97):
        p = bytes.fromhex(case["patterns_hex"][k])
        assert idx.count(p, faithful=True) == case["count"][k]


def test_batch_drivers_match_golden():
    case = load_golden("fm_100k.json")["cases"][0]
    idx = O.Index(golden_text(case["text"]), ssa_stride=32)
    pats = [bytes.fromhex(h) for h in case["patterns_hex"]]
    got = idx.count_batch(pats, nthreads=4)
    assert got.tolist() == case["count"]
    offs, pos = idx.locate_batch(pats, limit=case["limit"], nthreads=4)
    for q, loc in enumerate(case["locate"]):
        assert pos[offs[q]:offs[q + 1]].tolist() == loc["pos"]


@pytest.mark.parametrize("case", load_golden("bitvector.json")["cases"], ids=lambda c: c["name"])
def test_bitvector(case):
    n = case["n"]
    bits = np.unpackbits(np.frombuffer(bytes.fromhex(case["bits_hex"]), np.uint8),
                         bitorder="little")[:n]
    bv = O.BitVector(bits)
    assert bv.count_ones() == case["count_ones"]
    for i in range(n + 2):
        for faithful in (True, False):
            assert bv.rank1(i, faithful) == case["rank1"][i]
        assert bv.rank0(i) == case["rank0"][i]


def test_bitvector_from_words():
    """tests/bitvector_tests.cpp:186-202."""
    bv = O.BitVector(words=np.array([0xAAAAAAAAAAAAAAAA, 0x5555555555555555], np.uint64), nbits=128)
    assert bv.size() == 128 and bv.count_ones() == 64
    assert bv.rank1(64) == 32 and bv.rank1(128) == 64


@pytest.mark.parametrize("case", load_golden("wavelet.json")["cases"], ids=lambda c: c["name"])
def test_wavelet(case):
    seq = bytes.fromhex(case["seq_hex"])
    # the wavelet over an arbitrary sequence = the index's wavelet over a BWT equal to it
    idx = O.Index(bwt=seq)
    n = len(seq)
    for sym, ranks in case["rank"].items():
        c = int(sym)
        for i in range(n + 2):
            assert idx.wt_rank(c, i, faithful=(i % 7 == 0)) == ranks[i], (case["name"], c, i)
    assert [idx.wt_access(i) for i in range(n)] == case["access"]


def test_sa_doubling_equals_naive():
    """The doubling SA used for big fixtures equals sais.hpp's naive order."""
    rng = np.random.default_rng(3)
    for trial in range(60):
        n = int(rng.integers(0, 300))
        alpha = [b"ab", b"ACGT$", bytes(range(256)), b"a"][trial % 4]
        t = bytes(rng.choice(list(alpha), size=n).astype(np.uint8))
        assert O.sa_naive(t).tolist() == O.sa_doubling(t).tolist()


def test_synthetic_generators():
    """SURVEY §8(d) generators: terminator placement and alphabet."""
    d = O.gen_dna(42, 1000)
    assert d[-1] == ord("$") and set(d[:-1].tobytes()) <= set(b"ACGT")
    b = O.gen_bytes(42, 1000)
    assert b[-1] == 0 and b[:-1].min() >= 1
    q = O.gen_patterns_text(d, 20, 50, seed=4242)
    s = d.tobytes()
    assert all(bytes(p) in s for p in q)


@pytest.mark.parametrize("case", fm_golden_cases("fm_100k.json", "fm_1m.json"))
def test_reference_count_only_index(case):
    """bench.py's cpu_baseline of kind "reference": the reference's own
    FMIndex::count over BitVector tables built by the reference
    (oracle/ref/ref_shim.cpp ref_build_count_only) from the oracle's levels of the
    same BWT reproduces the golden counts of the genuine reference."""
    if O.ref_lib() is None:
        pytest.skip("oracle/_ref/libcs_ref.so not built (needs /root/reference)")
    text = golden_text(case["text"])
    idx = O.Index(text, ssa_stride=case["ssa_stride"])
    ref = O.RefCountIndex(O.Index(bwt=idx.bwt(), nthreads=2))
    pats = [bytes.fromhex(h) for h in case["patterns_hex"]]
    buf, offs = O.pack_patterns(pats)
    assert ref.count_batch(buf, offs, nthreads=4).tolist() == case["count"]


@pytest.mark.parametrize("case", fm_golden_cases("fm_kat.json", "fm_100k.json"))
def test_build_from_checked_sa(case):
    """orc_build_from_sa (the full-size tests' oracle: suffix array supplied, checked by
    orc_check_sa) answers every golden case exactly as the reference did."""
    text = golden_text(case["text"])
    if not text:
        pytest.skip("empty text: no suffix array to supply")
    sa = O.sa_doubling(text)
    assert O.check_suffix_array(text, sa)
    idx = O.Index(text, ssa_stride=case["ssa_stride"], sa=sa, nthreads=3)
    pats = [bytes.fromhex(h) for h in case["patterns_hex"]]
    assert [idx.count(p) for p in pats] == case["count"]
    for p, loc in zip(pats, case["locate"]):
        if "pos" in loc:
            assert idx.locate(p, limit=case["limit"]) == loc["pos"]


def test_check_suffix_array_rejects():
    rng = np.random.default_rng(3)
    for t in (b"banana$", b"aaaa", b"abab", b"x", O.gen_dna(9, 3000).tobytes(),
              bytes(rng.integers(0, 256, 2000).astype(np.uint8))):
        sa = O.sa_naive(t)
        assert O.check_suffix_array(t, sa)
        if len(t) > 1:
            sw = sa.copy()
            i = int(rng.integers(0, len(t) - 1))
            sw[[i, i + 1]] = sw[[i + 1, i]]
            assert not O.check_suffix_array(t, sw)
            dup = sa.copy()
            dup[0] = dup[-1]
            assert not O.check_suffix_array(t, dup)
        assert not O.check_suffix_array(t, sa[:-1])
        big = sa.copy()
        big[0] = len(t)
        assert not O.check_suffix_array(t, big)


@pytest.mark.parametrize("fname", ["fm_100k.json", "fm_1m.json"])
def test_scan_count_matches_reference(fname):
    """The index-free scan (orc_scan_count, the full-size checker of test_gpu_scale.py)
    against the genuine reference's counts and positions (row order sorted = text order):
    every fixture case with a unique smallest terminator, grouped by pattern length."""
    for case in load_golden(fname)["cases"]:
        text = golden_text(case["text"])
        t = np.frombuffer(text, np.uint8)
        if not (t[-1] < t[:-1]).all():
            continue  # the scan equals count() only with a unique smallest terminator
        pats = [bytes.fromhex(h) for h in case["patterns_hex"]]
        for m in sorted(set(len(p) for p in pats)):
            sel = [q for q, p in enumerate(pats) if len(p) == m and p]
            P = np.frombuffer(b"".join(pats[q] for q in sel), np.uint8).reshape(len(sel), m)
            cnt, offs, pos = O.scan_count(t, P, nloc=len(sel), nthreads=4)
            assert cnt.tolist() == [case["count"][q] for q in sel], (fname, m)
            for k, q in enumerate(sel):
                want = sorted(case["locate"][q]["pos"]) if case["count"][q] <= case["limit"] else None
                if want is not None:
                    assert pos[offs[k]:offs[k + 1]].tolist() == want, (fname, m, q)


def test_scan_count_edge_cases():
    t = np.frombuffer(b"abababab$", np.uint8)
    P = np.frombuffer(b"abaab$ba", np.uint8).reshape(4, 2)  # ab, aa, b$, ba
    cnt, offs, pos = O.scan_count(t, P, nloc=4, nthreads=3)
    assert cnt.tolist() == [4, 0, 1, 3]
    assert pos.tolist() == [0, 2, 4, 6, 7, 1, 3, 5] and offs.tolist() == [0, 4, 4, 5, 8]
    # duplicates share one count; windows at both ends; more threads than windows
    P = np.frombuffer(b"abb$abb$", np.uint8).reshape(4, 2)
    assert O.scan_count(t, P, nthreads=16).tolist() == [4, 1, 4, 1]
    assert O.scan_count(t, np.frombuffer(b"abababab$x", np.uint8).reshape(1, 10)).tolist() == [0]
    # rdna: heavy repeats, the index and the scan agree on every Q_text 20-mer
    r = O.gen_rdna(42, 300_000)
    idx = O.Index(r)
    Q = O.gen_patterns_text(r, 20, 3000, seed=4242)
    assert np.array_equal(O.scan_count(r, Q, nthreads=8), idx.count_batch([bytes(p) for p in Q]))
    # and on a σ = 256 text, 8-mers and 3-mers (many hits)
    b = O.gen_bytes(7, 200_000)
    ib = O.Index(b)
    for m in (8, 3, 1):
        Q = O.gen_patterns_text(b, m, 2000, seed=11)
        assert np.array_equal(O.scan_count(b, Q, nthreads=8), ib.count_batch([bytes(p) for p in Q]))
