"""CSIDX, the reference's single-file index format (src/serialization/serialization.hpp:1-83,
writer serialization.cpp:26-147, reader :153-335), read and written over the C ABI
(csrc/fm_csidx.cpp).

The reference's writer never finishes a file (IndexWriter::align_to does not advance,
serialization.cpp:44-54) and FMIndex never calls it, so no reference-written CSIDX exists.
The layout is pinned against the reference's own READER instead (round 4): files written by
cs_csidx_write (the host writer cs_fm_save_csidx uses too) from the oracle's members (the
ones build_from_text leaves, fm_index.cpp:36-66) are opened by the genuine cs::IndexReader
(serialization.cpp:153-335, compiled into oracle/_ref/libcs_ref.so by `make -C oracle ref`),
whose getters must return exactly those members; the GPU test then checks that a device
index's save_csidx writes the same bytes.  Files written by `write_csidx` below (the
documented layout in Python) exercise the reader's validation.
"""
import os
import struct

import numpy as np
import pytest

import oracle as O
from conftest import load_pkg

FOOTER = 0x444E4553435300


def _pad(buf: bytearray):
    buf.extend(b"\0" * ((8 - len(buf) % 8) % 8))


def write_csidx(path, bwt: bytes, ssa, stride: int, text: bytes | None = None, C=None,
                magic=b"CSIDX\0\0\0", version=1, text_len=None, ssa_count=None):
    """IndexHeader (88 B) + text / bwt / C / ssa sections + footer, each 8-B aligned."""
    offs = [0] * 8
    body = bytearray(88)
    if text is not None:
        offs[1] = len(body)
        body += struct.pack("<Q", len(text)) + text
        _pad(body)
    offs[2] = len(body)
    body += struct.pack("<Q", len(bwt)) + bwt
    _pad(body)
    if C is not None:
        offs[3] = len(body)
        body += struct.pack("<Q", len(C)) + np.asarray(C, np.uint32).tobytes()
        _pad(body)
    offs[4] = len(body)
    s = np.asarray(ssa, np.uint32)
    body += struct.pack("<I", stride)
    _pad(body)
    body += struct.pack("<Q", len(s) if ssa_count is None else ssa_count) + s.tobytes()
    _pad(body)
    offs[7] = len(body)
    body += struct.pack("<Q", FOOTER)
    body[:88] = magic + struct.pack("<HHIQ", version, 0, 0,
                                    len(bwt) if text_len is None else text_len) + \
        struct.pack("<8Q", *offs)
    with open(path, "wb") as f:
        f.write(bytes(body))


def read_csidx(path):
    """The documented layout back into (text, bwt, C, stride, ssa)."""
    b = open(path, "rb").read()
    assert b[:5] == b"CSIDX"
    ver, _, _, n = struct.unpack_from("<HHIQ", b, 8)
    offs = struct.unpack_from("<8Q", b, 24)
    assert ver == 1 and all(o % 8 == 0 for o in offs)

    def arr(off, dt):
        (k,) = struct.unpack_from("<Q", b, off)
        return np.frombuffer(b, dt, k, off + 8)

    text = arr(offs[1], np.uint8).tobytes() if offs[1] else None
    bwt = arr(offs[2], np.uint8).tobytes()
    C = arr(offs[3], np.uint32) if offs[3] else None
    (stride,) = struct.unpack_from("<I", b, offs[4])
    ssa = arr(offs[4] + 8, np.uint32)
    assert struct.unpack_from("<Q", b, offs[7])[0] == FOOTER and n == len(bwt)
    return text, bwt, C, stride, ssa


TEXTS = {
    "banana": b"banana$",
    "mississippi": b"mississippi$",
    "dna_5k": O.gen_dna(3, 5000).tobytes() + b"$",
    "bytes_4k": O.gen_bytes(5, 4000).tobytes() + b"\0",
}


def _arrays(t, stride=16):
    o = O.Index(t, ssa_stride=stride)
    return o, o.bwt().tobytes(), o.ssa(), np.asarray(o.C(), np.uint64)


# ---- CPU: the writer against the reference's own reader ------------------------------

REF_READS = pytest.mark.skipif(not (O.ref_lib() is not None and hasattr(O.ref_lib(), "ref_csidx_open")),
                               reason="oracle/_ref/libcs_ref.so (make -C oracle ref) not built")


@REF_READS
@pytest.mark.parametrize("name", sorted(TEXTS) + ["dna_100k"])
@pytest.mark.parametrize("with_text", [False, True])
@pytest.mark.parametrize("stride", [1, 7, 32])
def test_writer_vs_reference_reader(tmp_path, name, with_text, stride):
    """cs_csidx_write's file through cs::IndexReader (the reference's mmap reader): header
    magic / version accepted (serialization.cpp:171-174), text_len, and every section the
    getters return — get_text, get_bwt, get_c_array (C_, 257 x u32), get_ssa with its stride
    — equal to the oracle's members; our own reader agrees (cs_csidx_check)."""
    pkg = load_pkg()
    t = TEXTS[name] if name in TEXTS else O.gen_dna(8, 99_999).tobytes()
    o, bwt, ssa, C = _arrays(t, stride)
    p = str(tmp_path / "w.csidx")
    pkg.csidx_write(p, bwt, ssa, stride, t if with_text else None)
    r = O.ref_read_csidx(p)
    assert r["version"] == 1 and r["text_len"] == len(t)
    assert r["bwt"].tobytes() == bwt
    assert np.array_equal(r["C"], C.astype(np.uint32))
    assert r["stride"] == stride and np.array_equal(r["ssa"], ssa.astype(np.uint32))
    assert (r["text"].tobytes() if r["text"] is not None else None) == (t if with_text else None)
    assert pkg.csidx_check(p) == {"n": len(t), "ssa_stride": stride, "has_text": with_text}
    # the Python restatement of the layout writes the same bytes
    q = str(tmp_path / "py.csidx")
    write_csidx(q, bwt, ssa, stride, t if with_text else None, C=C.astype(np.uint32))
    assert open(p, "rb").read() == open(q, "rb").read()


@REF_READS
def test_reference_reader_rejects_what_we_reject(tmp_path):
    """A bad magic is refused by both readers with the reference's message."""
    pkg = load_pkg()
    o, bwt, ssa, C = _arrays(TEXTS["banana"], 4)
    p = str(tmp_path / "bad.csidx")
    write_csidx(p, bwt, ssa, 4, magic=b"CSIDY\0\0\0")
    with pytest.raises(RuntimeError, match="Invalid index file: bad magic or version"):
        O.ref_read_csidx(p)
    with pytest.raises(RuntimeError, match="bad magic or version"):
        pkg.csidx_check(p)


def test_writer_rejects_bad_arrays(tmp_path):
    pkg = load_pkg()
    o, bwt, ssa, C = _arrays(TEXTS["banana"], 4)
    with pytest.raises(RuntimeError, match="ceil"):
        pkg.csidx_write(str(tmp_path / "x.csidx"), bwt, ssa[:-1], 4)
    with pytest.raises(RuntimeError, match="ceil"):
        pkg.csidx_write(str(tmp_path / "x.csidx"), bwt, ssa, 0)


# ---- CPU: the reader's validation (no device) -----------------------------------


@pytest.mark.parametrize("name", sorted(TEXTS))
@pytest.mark.parametrize("with_text", [False, True])
def test_check_valid(tmp_path, name, with_text):
    t = TEXTS[name]
    _, bwt, ssa, C = _arrays(t)
    p = str(tmp_path / "x.csidx")
    write_csidx(p, bwt, ssa, 16, text=t if with_text else None, C=C)
    assert load_pkg().csidx_check(p) == {"n": len(t), "ssa_stride": 16, "has_text": with_text}


BAD = {
    "magic": (dict(magic=b"CSIDY\0\0\0"), "bad magic or version"),  # serialization.cpp:174
    "version": (dict(version=2), "bad magic or version"),
    "text_len": (dict(text_len=5), "text_len differs"),
    "ssa_count": (dict(ssa_count=2), r"ceil\(n / stride\)"),
    "C": (dict(C="bad"), "C array does not match"),
    "text": (dict(text=b"short"), "text section"),
    "sample": (dict(ssa="bad"), "SSA sample past the text"),
}


@pytest.mark.parametrize("what", sorted(BAD))
def test_check_rejects(tmp_path, what):
    t = TEXTS["mississippi"]
    _, bwt, ssa, C = _arrays(t, 4)
    kw, msg = BAD[what]
    kw = dict(kw)
    if kw.get("C") == "bad":
        kw["C"] = C.copy()
        kw["C"][3] += 1
    if isinstance(kw.get("ssa"), str):
        ssa = ssa.copy()
        ssa[1] = len(t)
        kw.pop("ssa")
    p = str(tmp_path / "bad.csidx")
    write_csidx(p, bwt, ssa, 4, C=kw.pop("C", C), **kw)
    with pytest.raises(RuntimeError, match=msg):
        load_pkg().csidx_check(p)


def test_check_truncated_and_missing(tmp_path):
    pkg = load_pkg()
    t = TEXTS["banana"]
    _, bwt, ssa, C = _arrays(t, 2)
    p = str(tmp_path / "t.csidx")
    write_csidx(p, bwt, ssa, 2, C=C)
    b = open(p, "rb").read()
    open(p, "wb").write(b[:60])
    with pytest.raises(RuntimeError, match="too small"):
        pkg.csidx_check(p)
    open(p, "wb").write(b[:-30])  # the SSA runs past the end of the file
    with pytest.raises(RuntimeError, match="SSA"):
        pkg.csidx_check(p)
    with pytest.raises(RuntimeError, match="cannot open"):
        pkg.csidx_check(str(tmp_path / "absent.csidx"))


# ---- GPU: open / save through the engine ----------------------------------------


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(TEXTS))
def test_open_csidx(tmp_path, name):
    """A CSIDX file of the reference's members opens as an index answering as the oracle
    does (count / locate / extract), through open_csidx and open_directory alike."""
    import torch  # noqa: F401  (one HIP runtime in the process)
    pkg = load_pkg()
    t = TEXTS[name]
    o, bwt, ssa, C = _arrays(t)
    p = str(tmp_path / "i.csidx")
    write_csidx(p, bwt, ssa, 16, text=t, C=C)
    rng = np.random.default_rng(len(t))
    pats = [t[i:i + k] for i, k in zip(rng.integers(0, max(1, len(t) - 8), 200),
                                       rng.integers(1, 9, 200))] + [b"", b"\xfe\xfd"]
    want = [o.count(q) for q in pats]
    for g in (pkg.FMIndex.open_csidx(p), pkg.FMIndex.open_directory(p)):
        assert g.n == len(t) and g.info().ssa_stride == 16
        assert g.count_batch(pats).tolist() == want
        for q in pats[:40]:
            try:
                w = o.locate(q, limit=50)
            except RuntimeError as e:
                with pytest.raises(RuntimeError) as ei:
                    g.locate(q, limit=50)
                assert str(ei.value) == str(e)
                continue
            assert g.locate(q, limit=50) == w
        assert g.extract(1, 5) == t[1:6]
    # without the text section: the index answers, extract is unsupported
    write_csidx(p, bwt, ssa, 16, C=None)
    g = pkg.FMIndex.open_csidx(p)
    assert g.count_batch(pats).tolist() == want
    with pytest.raises(RuntimeError):
        g.extract(1, 5)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["mississippi", "dna_5k", "bytes_4k"])
def test_save_csidx_round_trip(tmp_path, name):
    """save_csidx writes the reference's members (the BWT, ssa_ at the index's stride,
    C_, the text) in the documented layout; opening it again gives the same answers."""
    import torch  # noqa: F401
    pkg = load_pkg()
    t = TEXTS[name]
    g = pkg.FMIndex.build_from_text(t)
    p = str(tmp_path / "s.csidx")
    g.save_csidx(p)
    stride = g.info().ssa_stride
    o = O.Index(t, ssa_stride=stride)
    text, bwt, C, st, ssa = read_csidx(p)
    assert text == t and bwt == o.bwt().tobytes() and st == stride
    # the bytes the host writer (pinned against cs::IndexReader on the CPU) writes for the
    # oracle's members
    q = str(tmp_path / "host.csidx")
    pkg.csidx_write(q, o.bwt().tobytes(), o.ssa(), stride, t)
    assert open(p, "rb").read() == open(q, "rb").read()
    assert np.array_equal(ssa, o.ssa().astype(np.uint32))
    assert np.array_equal(C, np.asarray(o.C(), np.uint32))
    assert pkg.csidx_check(p) == {"n": len(t), "ssa_stride": stride, "has_text": True}
    h = pkg.FMIndex.open_csidx(p)
    rng = np.random.default_rng(7)
    pats = [t[i:i + k] for i, k in zip(rng.integers(0, len(t) - 8, 200), rng.integers(1, 12, 200))]
    assert h.count_batch(pats).tolist() == g.count_batch(pats).tolist()
    a, b = g.locate_batch(pats, limit=20), h.locate_batch(pats, limit=20)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert h.extract(2, 6) == t[2:8]
