"""Device-pointer entry points (the *_device forms of include/cs_fmindex.h) against
their host-buffer twins and the text: count, locate ranges + walk, extract."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import load_pkg

pytestmark = pytest.mark.gpu


def _dev(a, dtype):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dtype).cuda()


@pytest.mark.parametrize("kind", ["dna", "bytes"])
def test_device_forms_match_host(kind):
    pkg = load_pkg()
    st = torch.cuda.current_stream().cuda_stream
    t = (O.gen_dna(5, 100_000) if kind == "dna" else O.gen_bytes(5, 100_000)).tobytes()
    n = len(t)
    g = pkg.FMIndex.build_from_text(t)
    m = 12 if kind == "dna" else 4
    P = O.gen_patterns_text(np.frombuffer(t, np.uint8), m, 3000)
    buf = P.reshape(-1)
    offs = np.arange(0, (len(P) + 1) * m, m, dtype=np.uint64)
    want = g.count_batch(buf=buf, offs=offs)
    d_p, d_o = _dev(buf, torch.uint8), _dev(offs.astype(np.int64), torch.int64)
    d_c = torch.empty(len(P), dtype=torch.int64, device="cuda")
    g.count_batch_device(d_p.data_ptr(), d_o.data_ptr(), len(P), d_c.data_ptr(), st)
    torch.cuda.synchronize()
    assert d_c.cpu().numpy().astype(np.uint64).tolist() == want.tolist()
    # locate: ranges + walk == host locate_batch
    lo, lp = g.locate_batch(buf=buf, offs=offs, limit=7)
    d_sp = torch.empty(len(P), dtype=torch.int64, device="cuda")
    d_oo = torch.empty(len(P) + 1, dtype=torch.int64, device="cuda")
    tot = g.locate_ranges_device(d_p.data_ptr(), d_o.data_ptr(), len(P), 7, d_sp.data_ptr(),
                                 d_oo.data_ptr(), st)
    d_pos = torch.empty(max(tot, 1), dtype=torch.int64, device="cuda")
    g.locate_walk_device(d_sp.data_ptr(), d_oo.data_ptr(), len(P), tot, d_pos.data_ptr(), st)
    torch.cuda.synchronize()
    assert d_oo.cpu().numpy().astype(np.uint64).tolist() == np.asarray(lo).tolist()
    assert d_pos[:tot].cpu().numpy().astype(np.uint64).tolist() == np.asarray(lp).tolist()
    # extract: clamped slices, including pos >= n and tails
    rng = np.random.default_rng(3)
    pos = np.concatenate([rng.integers(0, n, 2000), [n - 1, n - 5, n, n + 3, 0]]).astype(np.int64)
    ln = np.concatenate([rng.integers(0, 60, 2000), [10, 10, 4, 4, 0]]).astype(np.int64)
    clamped = np.where(pos < n, np.minimum(ln, n - np.minimum(pos, n)), 0)
    oo = np.concatenate([[0], np.cumsum(clamped)]).astype(np.int64)
    d_out = torch.empty(max(int(oo[-1]), 1), dtype=torch.uint8, device="cuda")
    d_pos_x, d_len_x, d_oo_x = (_dev(pos, torch.int64), _dev(ln, torch.int64),
                                _dev(oo, torch.int64))  # kept alive across the launch
    g.extract_device(d_pos_x.data_ptr(), d_len_x.data_ptr(), d_oo_x.data_ptr(), len(pos),
                     d_out.data_ptr(), st)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy().tobytes()
    for q in range(len(pos)):
        assert out[oo[q]:oo[q + 1]] == t[pos[q]:pos[q] + ln[q]], q


def test_concurrent_calls_share_nothing_mutable():
    """The handle is immutable after creation and safe from several host threads
    (SURVEY §8(b)): count / locate from 8 threads at once, on an index whose LF walk
    overruns for some patterns (no terminator) and not for others, give each call its
    serial result or its own overrun error."""
    import threading
    pkg = load_pkg()
    rng0 = np.random.default_rng(1)  # no terminator: some LF walks cycle (overrun)
    t = bytes(rng0.choice(list(b"ab"), 300).astype(np.uint8))
    g = pkg.FMIndex.build_from_text(t, pkg.BuildParams(ssa_stride=8))
    o = O.Index(t, ssa_stride=8)
    pats = sorted({t[i:i + k] for i in range(0, 200, 7) for k in (1, 2, 3, 5)})
    serial = {}
    for p in pats:
        try:
            serial[p] = ("ok", o.locate(p, limit=20), o.count(p))
        except RuntimeError as e:
            serial[p] = ("err", str(e), o.count(p))
    assert any(v[0] == "err" for v in serial.values()) and any(v[0] == "ok" for v in serial.values())
    bad = []

    def worker(seed):
        rng = np.random.default_rng(seed)
        for _ in range(60):
            p = pats[rng.integers(len(pats))]
            kind, want, cnt = serial[p]
            if g.count(p) != cnt:
                bad.append(("count", p))
            try:
                got = g.locate(p, limit=20)
                if kind != "ok" or got != want:
                    bad.append(("locate", p))
            except RuntimeError as e:
                if kind != "err" or str(e) != want:
                    bad.append(("error", p))

    th = [threading.Thread(target=worker, args=(s,)) for s in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not bad, bad[:5]


def test_null_pattern_pointer():
    """A device batch of empty patterns may pass d_pats = NULL (count("") = n, locate("") =
    {}, fm_index.cpp:80, :109); with a non-empty pattern a NULL d_pats is CS_ERR_INVALID
    (ADVICE r03)."""
    pkg = load_pkg()
    t = O.gen_dna(4, 5000).tobytes()
    g = pkg.FMIndex.build_from_text(t)
    st = torch.cuda.current_stream().cuda_stream
    for offs, ok in (([7, 7, 7, 7], True), ([0, 0, 3, 3], False)):
        d_o = _dev(np.array(offs, np.int64), torch.int64)
        d_c = torch.full((3,), -1, dtype=torch.int64, device="cuda")
        if ok:
            g.count_batch_device(0, d_o.data_ptr(), 3, d_c.data_ptr(), st)
            torch.cuda.synchronize()
            assert d_c.cpu().tolist() == [len(t)] * 3
            d_oo = torch.full((4,), -1, dtype=torch.int64, device="cuda")
            tot, done = g.locate_device(0, d_o.data_ptr(), 3, 10, d_oo.data_ptr(), 0, 0, st)
            assert done and tot == 0 and d_oo.cpu().tolist() == [0, 0, 0, 0]
        else:
            with pytest.raises(RuntimeError, match="null batch pointer"):
                g.count_batch_device(0, d_o.data_ptr(), 3, d_c.data_ptr(), st)
            d_oo = torch.zeros(4, dtype=torch.int64, device="cuda")
            with pytest.raises(RuntimeError, match="null batch pointer"):
                g.locate_device(0, d_o.data_ptr(), 3, 10, d_oo.data_ptr(), 0, 0, st)


def test_long_routing_concurrent_streams():
    """Long-pattern routing inside the call (fm_device.hpp LongList): the
    staged kernel lists the patterns its one read cannot answer and k_count_long /
    k_locate_long take them from the call's own lists — no state in the handle.  4 host
    threads, each on its own stream, alternate short-only, long-only and mixed device batches
    (counts, and locates in one call) on one handle: every result equals the oracle's."""
    import threading
    pkg = load_pkg()
    t = O.gen_dna(9, 400_000)
    g = pkg.FMIndex.build_from_text(t.tobytes())
    if not g.info().packed_text_bytes:
        pytest.skip("no long-pattern kernels on this index")
    o = O.Index(t)
    rng = np.random.default_rng(2)
    batches = []
    for kind in ("short", "long", "mixed", "mixed_sparse"):
        pats = []
        for _ in range(3000):
            if kind == "short" or (kind == "mixed_sparse" and rng.random() < 0.97):
                m = int(rng.integers(1, 32))
            elif kind == "long":
                m = int(rng.integers(32, 160))
            else:
                m = int(rng.integers(1, 160))
            i = int(rng.integers(0, len(t) - m))
            p = bytearray(t[i:i + m].tobytes())
            if rng.random() < 0.3:
                p[int(rng.integers(0, m))] = b"ACGT"[int(rng.integers(0, 4))]
            pats.append(bytes(p))
        buf, offs = O.pack_patterns(pats)
        woffs, wpos = o.locate_batch(buf=buf, offs=offs, limit=50, nthreads=8)
        batches.append((buf, offs, o.count_batch(buf=buf, offs=offs, nthreads=8), woffs, wpos))
    bad = []

    def worker(seed):
        rng_w = np.random.default_rng(seed)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for it in range(24):
                buf, offs, want, woffs, wpos = batches[int(rng_w.integers(len(batches)))]
                npat = len(offs) - 1
                d_p, d_o = _dev(buf, torch.uint8), _dev(offs.astype(np.int64), torch.int64)
                d_c = torch.empty(npat, dtype=torch.int64, device="cuda")
                g.count_batch_device(d_p.data_ptr(), d_o.data_ptr(), npat, d_c.data_ptr(), s.cuda_stream)
                d_oo = torch.empty(npat + 1, dtype=torch.int64, device="cuda")
                d_pos = torch.empty(max(int(woffs[-1]), 1), dtype=torch.int64, device="cuda")
                tot, ok = g.locate_device(d_p.data_ptr(), d_o.data_ptr(), npat, 50, d_oo.data_ptr(),
                                          d_pos.data_ptr(), d_pos.numel(), s.cuda_stream)
                s.synchronize()
                if not np.array_equal(d_c.cpu().numpy().astype(np.uint64), want):
                    bad.append(("count", seed, it))
                if not (ok and tot == woffs[-1] and
                        np.array_equal(d_oo.cpu().numpy().astype(np.uint64), woffs) and
                        np.array_equal(d_pos[:tot].cpu().numpy().astype(np.uint64), wpos)):
                    bad.append(("locate", seed, it))

    th = [threading.Thread(target=worker, args=(sd,)) for sd in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not bad, bad[:5]


@pytest.mark.parametrize("engine", ["auto", "qwm", "wavelet", "learned", "records", "records16"])
def test_export_import_image(engine, build_opts):
    """The device image (cs_fm_export_meta/_parts -> cs_fm_import): the copy answers
    count / locate / extract exactly as the original (context records and the full
    suffix array included)."""
    if engine in ("records", "records16"):
        build_opts(CS_FM_CTX_RECORDS="1" if engine == "records" else "16")
    elif engine != "auto":
        build_opts(CS_FM_ENGINE=engine)
    pkg = load_pkg()
    t = O.gen_dna(9, 50_000).tobytes()
    g = pkg.FMIndex.build_from_text(t)
    meta, sizes = g.export_meta()
    assert meta.startswith(b"format cs_fmindex/") and len(sizes) >= 4
    parts = [torch.empty(max(b, 1), dtype=torch.uint8, device="cuda") for b in sizes]
    g.export_parts([p.data_ptr() for p in parts])
    torch.cuda.synchronize()
    c = pkg.FMIndex.import_image(meta, [p.data_ptr() for p in parts], 0)
    del parts
    assert c.info().engine == g.info().engine and c.info().walk_marks == g.info().walk_marks
    assert c.info().context_q == g.info().context_q == {"auto": 7, "qwm": 8, "wavelet": 0, "learned": 7,
                                                        "records": 7, "records16": 7}[engine]
    assert c.info().prefix_bytes == g.info().prefix_bytes
    assert c.info().full_sa_bytes == g.info().full_sa_bytes == 4 * len(t)
    if engine in ("records", "records16"):
        rb = 32 if engine == "records" else 16
        assert c.info().record_bytes == g.info().record_bytes == rb
        assert g.info().prefix_bytes == rb * g.info().prefix_sigma ** g.info().prefix_k
    P = O.gen_patterns_text(np.frombuffer(t, np.uint8), 14, 500)
    pats = [bytes(r) for r in P] + [b"ACGTACGTAC", b"$", b""]
    assert c.count_batch(pats).tolist() == g.count_batch(pats).tolist()
    lo1, lp1 = g.locate_batch(pats, limit=9)
    lo2, lp2 = c.locate_batch(pats, limit=9)
    assert lo1.tolist() == lo2.tolist() and lp1.tolist() == lp2.tolist()
    assert c.extract_batch([0, 100, len(t) - 3], [10, 25, 10]) == [t[0:10], t[100:125], t[-3:]]


def test_host_batch_buffers_sharing_pages():
    """A large host batch whose pattern bytes and counts live in one caller arena (the
    counts start inside the patterns' last page): the pinned-copy path registers only
    whole inner pages, so neither copy is mistaken for pinned memory of the other."""
    pkg = load_pkg()
    t = O.gen_dna(5, 200_000).tobytes()
    g = pkg.FMIndex.build_from_text(t)
    P = O.gen_patterns_text(np.frombuffer(t, np.uint8), 20, 1_000_000, seed=9)
    npat = len(P)
    pb = npat * 20  # 20 MB, not a multiple of the page size
    start = (pb + 7) // 8 * 8
    arena = np.zeros(start + 8 * npat, np.uint8)
    arena[:pb] = P.reshape(-1)
    out = arena[start:].view(np.uint64)
    offs = np.arange(0, (npat + 1) * 20, 20, dtype=np.uint64)
    st = pkg.lib().cs_fm_count_batch(g._h, pkg._u8(arena), pkg._u64(offs), npat, pkg._u64(out), None)
    assert st == 0, pkg.lib().cs_fm_last_error()
    assert np.array_equal(out, g.count_batch(buf=P.reshape(-1), offs=offs))
    assert (out >= 1).all()


@pytest.mark.parametrize("chunk", [333_333, 1 << 20, 0])
def test_host_batch_chunked(chunk, build_opts):
    """cs_fm_count_batch over a large ragged host batch in chunks (CS_FM_HOST_CHUNK when the
    handle is created; 0 = the
    default 2 M patterns): the caller's pages page-locked piece by piece while earlier chunks
    run; offsets starting inside the caller's buffer (offs[0] > 0), empty patterns, the
    counts in the same arena right after the patterns — equal to one unchunked call."""
    pkg = load_pkg()
    t = O.gen_dna(6, 300_000).tobytes()
    if chunk:  # (read when the handle is created)
        build_opts(CS_FM_HOST_CHUNK=str(chunk))
    g = pkg.FMIndex.build_from_text(t)
    build_opts(CS_FM_HOST_CHUNK=str(10 ** 9))
    g1 = pkg.FMIndex.build_from_text(t)  # one chunk
    rng = np.random.default_rng(3)
    npat = 2_500_000
    lens = rng.integers(0, 33, npat)
    starts = rng.integers(0, len(t) - 40, npat)
    cols = np.arange(32)
    sel = (starts[:, None] + cols[None, :])[cols[None, :] < lens[:, None]]
    body = np.frombuffer(t, np.uint8)[sel].copy()
    body[rng.random(body.size) < 0.01] = ord("A")  # mutants: some absent
    lead = 4099
    start = (lead + body.size + 7) // 8 * 8
    arena = np.zeros(start + 8 * npat, np.uint8)
    arena[lead:lead + body.size] = body
    out = arena[start:].view(np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + lead
    st = pkg.lib().cs_fm_count_batch(g._h, pkg._u8(arena), pkg._u64(offs), npat, pkg._u64(out), None)
    assert st == 0, pkg.lib().cs_fm_last_error()
    want = g1.count_batch(buf=arena[:lead + body.size].copy(), offs=offs)
    assert np.array_equal(out, want)
    assert (out[lens == 0] == len(t)).all() and (out >= 1).mean() > 0.5


def test_host_batch_long_chunks(build_opts):
    """Host batches of long patterns take the long-pattern count kernel (CS_Q_LONG) chunk
    by chunk when every pattern of the chunk is longer than 96 characters; the chunk that
    holds a short pattern stays on the staged kernel — the oracle's counts either way."""
    pkg = load_pkg()
    t = O.gen_dna(8, 200_000).tobytes()
    g = pkg.FMIndex.build_from_text(t)
    ref = O.Index(t, ssa_stride=32)
    rng = np.random.default_rng(5)
    pats = []
    for i in range(3000):
        m = int(rng.integers(97, 200))
        s = int(rng.integers(0, len(t) - m - 1))
        p = bytearray(t[s:s + m])
        if i % 3 == 0:  # mutants: mostly absent
            p[int(rng.integers(0, m))] = ord("A")
        pats.append(bytes(p))
    pats[2500] = pats[2500][:20]
    want = [ref.count(p) for p in pats]
    build_opts(CS_FM_HOST_CHUNK="1000")  # (read when the handle is created)
    g = pkg.FMIndex.build_from_text(t)
    assert g.count_batch(pats).tolist() == want
    build_opts(CS_FM_HOST_CHUNK=str(10 ** 9))
    g = pkg.FMIndex.build_from_text(t)
    assert g.count_batch(pats[:2000]).tolist() == want[:2000]
    assert g.count_batch(pats).tolist() == want


@pytest.mark.parametrize("engine", ["auto", "qwm", "wavelet", "records16"])
def test_import_alloc_commit(engine, build_opts):
    """Replication without staging copies: the index's own part addresses
    (cs_fm_export_part_ptrs) copied into the parts of a handle allocated for them
    (cs_fm_import_alloc, then cs_fm_import_commit), through torch tensors over the raw
    device memory (shard.device_bytes) — the copy answers as the original."""
    if engine in ("records", "records16"):
        build_opts(CS_FM_CTX_RECORDS="1" if engine == "records" else "16")
    elif engine != "auto":
        build_opts(CS_FM_ENGINE=engine)
    pkg = load_pkg()
    import importlib
    shard = importlib.import_module("cs_fmindex_amd.shard")
    t = O.gen_dna(19, 40_000).tobytes()
    g = pkg.FMIndex.build_from_text(t)
    meta, sizes = g.export_meta()
    src = g.export_part_ptrs(len(sizes))
    c, dst = pkg.FMIndex.import_alloc(meta, len(sizes), 0)
    assert len(dst) == len(sizes) and all(dst)
    for s, d, nb in zip(src, dst, sizes):
        if nb:
            shard.device_bytes(d, nb, "cuda").copy_(shard.device_bytes(s, nb, "cuda"))
    c.import_commit()
    P = O.gen_patterns_text(np.frombuffer(t, np.uint8), 17, 400)
    pats = [bytes(r) for r in P] + [b"ACGTACGTAC", b"$", b""]
    assert c.count_batch(pats).tolist() == g.count_batch(pats).tolist()
    lo1, lp1 = g.locate_batch(pats, limit=9)
    lo2, lp2 = c.locate_batch(pats, limit=9)
    assert lo1.tolist() == lo2.tolist() and lp1.tolist() == lp2.tolist()


def _wire_reference(counts, cap):
    """The wire format of include/cs_fmindex.h (cs_counts_pack_wire), in numpy."""
    counts = np.asarray(counts, np.uint64)
    big = np.nonzero(counts >= 255)[0]
    hdr = np.array([len(big), cap], np.uint64)
    return hdr, set(zip(big.tolist(), counts[big].tolist())), np.minimum(counts, 255).astype(np.uint8)


@pytest.mark.parametrize("npat,cap", [(0, 4), (1, 4), (7, 4), (1001, 4), (100_003, 64), (100_003, 0)])
def test_counts_wire(npat, cap):
    """cs_counts_pack_wire writes the documented layout (u8 counts, every count >= 255 as
    one pair, the pair counter even past cap) and shard.unpack_counts restores the exact
    counts, or raises when the pairs did not fit."""
    pkg = load_pkg()
    import importlib
    shard = importlib.import_module("cs_fmindex_amd.shard")
    rng = np.random.default_rng(npat + cap)
    c = rng.integers(0, 300, npat).astype(np.int64)
    c[rng.random(npat) < 0.9] %= 255  # mostly small, some >= 255
    if npat > 3:
        c[3] = 4_000_000_000
    d = torch.from_numpy(c).cuda()
    nb = pkg.counts_wire_bytes(npat, cap)
    assert nb == 16 + 16 * cap + ((npat + 7) // 8) * 8
    wire = torch.full((nb,), 0xAB, dtype=torch.uint8, device="cuda")
    shard.pack_counts(pkg, d, wire, cap=cap)
    torch.cuda.synchronize()
    w = wire.cpu().numpy()
    hdr, pairs, u8 = _wire_reference(c, cap)
    assert w[:16].view(np.uint64).tolist() == hdr.tolist()
    got_pairs = w[16:16 + 16 * min(int(hdr[0]), cap)].view(np.uint64).reshape(-1, 2)
    assert set(map(tuple, got_pairs.tolist())) <= pairs and len(got_pairs) == min(int(hdr[0]), cap)
    assert w[16 + 16 * cap:16 + 16 * cap + npat].tolist() == u8.tolist()
    if hdr[0] <= cap:
        assert shard.unpack_counts(wire, npat).cpu().tolist() == c.tolist()
    else:
        with pytest.raises(OverflowError):
            shard.unpack_counts(wire, npat)


@pytest.mark.parametrize("chunk", [0, 300_000])
def test_concurrent_host_batches_share_pages(chunk, build_opts):
    """Two host threads count batches over the same large buffer at once — one the whole
    buffer, one a window starting inside it (overlapping registrations) — on distinct
    streams, in one piece or in chunks whose pages are registered piece by piece
    (CS_FM_HOST_CHUNK): the pin registry shares or bounces the pages, and both get the
    single-thread answer, repeatedly."""
    import threading
    if chunk:
        build_opts(CS_FM_HOST_CHUNK=str(chunk))
    pkg = load_pkg()
    t = O.gen_dna(23, 200_000).tobytes()
    g = pkg.FMIndex.build_from_text(t)
    m = 24
    P = O.gen_patterns_text(np.frombuffer(t, np.uint8), m, 1_200_000)  # 28.8 MB of patterns
    buf = np.ascontiguousarray(P.reshape(-1))
    offs = np.arange(0, (len(P) + 1) * m, m, dtype=np.uint64)
    want = g.count_batch(buf=buf, offs=offs)
    lo = 700_001  # window: patterns [lo, end) — its first page lies inside the first buffer
    res, errs = {}, []

    def run(key, o):
        try:
            for _ in range(4):
                res.setdefault(key, []).append(g.count_batch(buf=buf, offs=o).copy())
        except Exception as e:  # surfaced below
            errs.append(e)

    th = [threading.Thread(target=run, args=("all", offs)),
          threading.Thread(target=run, args=("win", offs[lo:]))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    assert all(np.array_equal(r, want) for r in res["all"])
    assert all(np.array_equal(r, want[lo:]) for r in res["win"])


@pytest.mark.parametrize("kind", ["dna", "bytes"])
def test_hbm_budget(kind, build_opts):
    """CS_FM_HBM_BUDGET: the optional structures are added in build order while the index
    fits; every budget answers count / locate / extract exactly as the default build, the
    footprint never exceeds max(budget, the base structures), and an ample budget builds
    the default index."""
    pkg = load_pkg()
    t = (O.gen_dna(21, 2_000_000) if kind == "dna" else O.gen_bytes(21, 1_000_000)).tobytes()
    m = 20 if kind == "dna" else 6
    P = O.gen_patterns_text(np.frombuffer(t, np.uint8), m, 20_000, seed=9)
    P = np.concatenate([P, O.gen_patterns_uniform(b"ACGT" if kind == "dna" else bytes(range(1, 256)),
                                                  m, 5_000, seed=10)])
    buf = P.reshape(-1)
    offs = np.arange(0, (len(P) + 1) * m, m, dtype=np.uint64)
    ref = pkg.FMIndex.build_from_text(t)
    want_c = ref.count_batch(buf=buf, offs=offs)
    want_l = ref.locate_batch(buf=buf[: 2000 * m], offs=offs[:2001], limit=50)
    full = int(sum(ref.export_meta()[1]))
    del ref
    sizes = []
    for budget in (1, full // 4, full // 2, (3 * full) // 4, full, 10 * full):
        build_opts(CS_FM_HBM_BUDGET=str(budget))
        g = pkg.FMIndex.build_from_text(t)
        nb = int(sum(g.export_meta()[1]))
        sizes.append(nb)
        assert g.count_batch(buf=buf, offs=offs).tolist() == want_c.tolist(), budget
        lo, lp = g.locate_batch(buf=buf[: 2000 * m], offs=offs[:2001], limit=50)
        assert np.asarray(lo).tolist() == np.asarray(want_l[0]).tolist(), budget
        assert np.asarray(lp).tolist() == np.asarray(want_l[1]).tolist(), budget
        assert g.extract(len(t) // 3, 40) == t[len(t) // 3: len(t) // 3 + 40]
        del g
    base = sizes[0]  # budget 1 B: the base structures only
    for budget, nb in zip((1, full // 4, full // 2, (3 * full) // 4, full, 10 * full), sizes):
        assert nb <= max(budget, base), (budget, nb, sizes)
    assert max(sizes) == sizes[-1] == full, sizes  # an ample budget builds the default index


def test_locate_one_call_many_tiles():
    """The one-call locate's tile scan over more tiles than one round of k_scan_tiles
    (> 32 k tiles of 512 patterns: 17 M patterns) equals the two-phase locate."""
    pkg = load_pkg()
    st = torch.cuda.current_stream().cuda_stream
    t = O.gen_dna(33, 200_000).tobytes()
    g = pkg.FMIndex.build_from_text(t)
    npat, m, lim = 17_000_000, 8, 3
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(5)
    acgt = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
    pats = acgt[torch.randint(0, 4, (npat * m,), device=dev, generator=gen)]
    offs = torch.arange(0, (npat + 1) * m, m, dtype=torch.int64, device=dev)
    oo1 = torch.empty(npat + 1, dtype=torch.int64, device=dev)
    pos1 = torch.empty(npat * lim, dtype=torch.int64, device=dev)
    tot1, ok = g.locate_device(pats.data_ptr(), offs.data_ptr(), npat, lim, oo1.data_ptr(),
                               pos1.data_ptr(), pos1.numel(), st)
    assert ok
    sp = torch.empty(npat, dtype=torch.int64, device=dev)
    oo2 = torch.empty(npat + 1, dtype=torch.int64, device=dev)
    tot2 = g.locate_ranges_device(pats.data_ptr(), offs.data_ptr(), npat, lim, sp.data_ptr(),
                                  oo2.data_ptr(), st)
    pos2 = torch.empty(max(tot2, 1), dtype=torch.int64, device=dev)
    g.locate_walk_device(sp.data_ptr(), oo2.data_ptr(), npat, tot2, pos2.data_ptr(), st)
    torch.cuda.synchronize()
    assert tot1 == tot2 and tot1 > 0
    assert torch.equal(oo1, oo2)
    assert torch.equal(pos1[:tot1], pos2[:tot2])
