"""oracle.py — ctypes front end of the C restatement (oracle/fm_oracle.c).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker or the timed CPU baseline,
never as the product path.  The product (the HIP library) never imports this.

Semantics follow the reference (citations in fm_oracle.c):
  count(p)          src/api/fm_index.cpp:79-101 (empty -> n, n==0 -> 0)
  locate(p, limit)  src/api/fm_index.cpp:107-157 (row order, limit, % n,
                    RuntimeError with the reference's message on overrun)
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libfm_oracle.so")
_lib = None

ORC_OK, ORC_ERR_LF_OVERRUN, ORC_ERR_SSA_RANGE, ORC_ERR_CAPACITY, ORC_ERR_NOSA = 0, 1, 2, 3, 4

_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)
_u16p = C.POINTER(C.c_uint16)
_vp = C.c_void_p


def build_lib() -> str:
    """Compile the restatement with gcc (oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", _HERE, "all"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
            os.path.join(_HERE, "fm_oracle.c")):
        build_lib()
    L = C.CDLL(_LIB_PATH)
    sig = {
        "orc_bv_build": (_vp, [_u8p, C.c_uint64]),
        "orc_bv_build_from_words": (_vp, [_u64p, C.c_uint64, C.c_uint64]),
        "orc_bv_free": (None, [_vp]),
        "orc_bv_size": (C.c_uint64, [_vp]),
        "orc_bv_rank1": (C.c_uint64, [_vp, C.c_uint64, C.c_int]),
        "orc_bv_rank0": (C.c_uint64, [_vp, C.c_uint64, C.c_int]),
        "orc_bv_count_ones": (C.c_uint64, [_vp]),
        "orc_bv_get": (C.c_uint8, [_vp, C.c_uint64]),
        "orc_bv_words": (_u64p, [_vp, _u64p]),
        "orc_bv_super": (_u64p, [_vp, _u64p]),
        "orc_bv_blocks": (_u16p, [_vp, _u64p]),
        "orc_sa_naive": (None, [_u8p, C.c_uint64, _u64p]),
        "orc_sa_doubling": (None, [_u8p, C.c_uint64, _u64p]),
        "orc_build": (_vp, [_u8p, C.c_uint64, C.c_uint32, C.c_int]),
        "orc_build_from_bwt": (_vp, [_u8p, C.c_uint64]),
        "orc_build_from_bwt_mt": (_vp, [_u8p, C.c_uint64, C.c_int]),
        "orc_build_from_sa": (_vp, [_u8p, C.c_uint64, _u64p, C.c_uint32, C.c_int]),
        "orc_check_sa": (C.c_int, [_u8p, C.c_uint64, _u64p, C.c_int]),
        "orc_free": (None, [_vp]),
        "orc_n": (C.c_uint64, [_vp]),
        "orc_ssa_stride": (C.c_uint32, [_vp]),
        "orc_get_sa": (None, [_vp, _u64p]),
        "orc_get_bwt": (None, [_vp, _u8p]),
        "orc_get_C": (None, [_vp, _u64p]),
        "orc_ssa_len": (C.c_uint64, [_vp]),
        "orc_get_ssa": (None, [_vp, _u64p]),
        "orc_level": (_vp, [_vp, C.c_int]),
        "orc_wt_rank": (C.c_uint64, [_vp, C.c_uint8, C.c_uint64, C.c_int]),
        "orc_wt_access": (C.c_uint8, [_vp, C.c_uint64, C.c_int]),
        "orc_lf": (C.c_uint64, [_vp, C.c_uint64, C.c_int]),
        "orc_count": (C.c_uint64, [_vp, _u8p, C.c_uint64, C.c_int]),
        "orc_locate": (C.c_int, [_vp, _u8p, C.c_uint64, C.c_uint64, _u64p, C.c_uint64, _u64p,
                                 C.c_int, _u64p]),
        "orc_extract": (C.c_uint64, [_vp, C.c_uint64, C.c_uint64, _u8p]),
        "orc_count_batch": (None, [_vp, _u8p, _u64p, C.c_uint64, _u64p, C.c_int, C.c_int, _u64p]),
        "orc_locate_batch": (C.c_int, [_vp, _u8p, _u64p, C.c_uint64, C.c_uint64, _u64p, _u64p,
                                       C.c_uint64, C.c_int, C.c_int]),
        "orc_attach_ssa": (None, [_vp, _u64p, C.c_uint64, C.c_uint32]),
        "orc_scan_count": (C.c_int, [_u8p, C.c_uint64, _u8p, C.c_uint64, C.c_uint64, _u64p,
                                     C.c_uint64, _u64p, _u64p, C.c_uint64, C.c_int]),
        "orc_gen_dna": (None, [C.c_uint64, C.c_uint64, _u8p]),
        "orc_gen_bytes": (None, [C.c_uint64, C.c_uint64, _u8p]),
        "orc_gen_rdna": (None, [C.c_uint64, C.c_uint64, _u8p]),
        "orc_gen_patterns_unif": (None, [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, _u8p]),
        "orc_gen_patterns_text": (None, [_u8p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                         _u8p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _u8(a: np.ndarray):
    return a.ctypes.data_as(_u8p)


def _u64(a: np.ndarray):
    return a.ctypes.data_as(_u64p)


def as_u8(x) -> np.ndarray:
    if isinstance(x, np.ndarray):
        return np.ascontiguousarray(x, dtype=np.uint8)
    if isinstance(x, str):
        x = x.encode("latin-1")
    return np.frombuffer(bytes(x), dtype=np.uint8).copy() if len(x) else np.zeros(0, np.uint8)


def pack_patterns(patterns) -> tuple[np.ndarray, np.ndarray]:
    """list of bytes -> (concatenated u8 bytes, u64 offsets[n+1])."""
    pats = [p.encode("latin-1") if isinstance(p, str) else bytes(p) for p in patterns]
    offs = np.zeros(len(pats) + 1, dtype=np.uint64)
    if pats:
        offs[1:] = np.cumsum([len(p) for p in pats], dtype=np.uint64)
    buf = np.frombuffer(b"".join(pats), dtype=np.uint8).copy() if offs[-1] else np.zeros(1, np.uint8)
    return buf, offs


# ---------------------------------------------------------------------------
class BitVector:
    """src/core/bitvector.{hpp,cpp} restated."""

    def __init__(self, bits=None, words=None, nbits=None):
        L = lib()
        if words is not None:
            w = np.ascontiguousarray(words, dtype=np.uint64)
            self._h = L.orc_bv_build_from_words(_u64(w), len(w), nbits)
        else:
            b = np.ascontiguousarray(bits, dtype=np.uint8)
            if len(b) == 0:
                b = np.zeros(1, np.uint8)
                self._h = L.orc_bv_build(_u8(b), 0)
            else:
                self._h = L.orc_bv_build(_u8(b), len(b))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_bv_free(self._h)
            self._h = None

    def size(self):
        return lib().orc_bv_size(self._h)

    def rank1(self, i, faithful=True):
        return lib().orc_bv_rank1(self._h, i, int(faithful))

    def rank0(self, i, faithful=True):
        return lib().orc_bv_rank0(self._h, i, int(faithful))

    def count_ones(self):
        return lib().orc_bv_count_ones(self._h)

    def get(self, i):
        return lib().orc_bv_get(self._h, i)


class LevelView:
    """Borrowed view of one wavelet level (owned by the index)."""

    def __init__(self, h, owner):
        self._h, self._owner = h, owner

    def rank1(self, i, faithful=False):
        return lib().orc_bv_rank1(self._h, i, int(faithful))

    def size(self):
        return lib().orc_bv_size(self._h)

    def words_ptr(self):
        """(address, count) of the packed words, borrowed from the owning index."""
        n = C.c_uint64()
        w = lib().orc_bv_words(self._h, C.byref(n))
        return C.cast(w, C.c_void_p).value, n.value

    def tables(self):
        L = lib()
        n = C.c_uint64()
        w = L.orc_bv_words(self._h, C.byref(n))
        words = np.ctypeslib.as_array(w, shape=(n.value,)).copy() if n.value else np.zeros(0, np.uint64)
        s = L.orc_bv_super(self._h, C.byref(n))
        sup = np.ctypeslib.as_array(s, shape=(n.value,)).copy() if n.value else np.zeros(0, np.uint64)
        b = L.orc_bv_blocks(self._h, C.byref(n))
        blk = np.ctypeslib.as_array(b, shape=(n.value,)).copy() if n.value else np.zeros(0, np.uint16)
        return words, sup, blk


class Index:
    """cs::FMIndex restated (src/api/fm_index.{hpp,cpp})."""

    def __init__(self, text=None, ssa_stride=32, sa_algo=0, bwt=None, nthreads=1, sa=None):
        """From the text (suffix sort here), from a BWT (count only), or from the text and
        a suffix array the caller has checked (check_suffix_array): no sort."""
        L = lib()
        if sa is not None:
            t = as_u8(text)
            sa64 = np.ascontiguousarray(sa, np.uint64)
            assert len(sa64) == len(t) and len(t) > 0
            self._h = L.orc_build_from_sa(_u8(t), len(t), _u64(sa64), ssa_stride, nthreads)
        elif bwt is not None:
            b = as_u8(bwt)
            self._h = L.orc_build_from_bwt_mt(_u8(b) if len(b) else _u8(np.zeros(1, np.uint8)),
                                             len(b), nthreads)
        else:
            t = as_u8(text)
            tt = t if len(t) else np.zeros(1, np.uint8)
            self._h = L.orc_build(_u8(tt), len(t), ssa_stride, sa_algo)
        self.n = L.orc_n(self._h)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_free(self._h)
            self._h = None

    # structures -----------------------------------------------------------
    def sa(self):
        out = np.zeros(max(self.n, 1), np.uint64)
        lib().orc_get_sa(self._h, _u64(out))
        return out[: self.n]

    def bwt(self):
        out = np.zeros(max(self.n, 1), np.uint8)
        lib().orc_get_bwt(self._h, _u8(out))
        return out[: self.n]

    def C(self):
        out = np.zeros(257, np.uint64)
        lib().orc_get_C(self._h, _u64(out))
        return out

    def ssa(self):
        k = lib().orc_ssa_len(self._h)
        out = np.zeros(max(k, 1), np.uint64)
        lib().orc_get_ssa(self._h, _u64(out))
        return out[:k]

    def ssa_stride(self):
        return lib().orc_ssa_stride(self._h)

    def level(self, l):
        return LevelView(lib().orc_level(self._h, l), self)

    def wt_rank(self, c, i, faithful=False):
        return lib().orc_wt_rank(self._h, c, i, int(faithful))

    def wt_access(self, i, faithful=False):
        return lib().orc_wt_access(self._h, i, int(faithful))

    def lf(self, i, faithful=False):
        return lib().orc_lf(self._h, i, int(faithful))

    # queries --------------------------------------------------------------
    def count(self, p, faithful=False):
        b = as_u8(p)
        bb = b if len(b) else np.zeros(1, np.uint8)
        return lib().orc_count(self._h, _u8(bb), len(b), int(faithful))

    def locate(self, p, limit=100000, faithful=False):
        b = as_u8(p)
        bb = b if len(b) else np.zeros(1, np.uint8)
        cap = max(1, min(limit, self.n))
        out = np.zeros(cap, np.uint64)
        nout = C.c_uint64()
        aux = np.zeros(2, np.uint64)
        st = lib().orc_locate(self._h, _u8(bb), len(b), limit, _u64(out), cap, C.byref(nout),
                              int(faithful), _u64(aux))
        if st == ORC_ERR_LF_OVERRUN:
            raise RuntimeError("locate: LF walk exceeded text length")
        if st == ORC_ERR_SSA_RANGE:
            raise RuntimeError("locate: SSA sample index out of range: idx=%d, size=%d"
                               % (aux[0], aux[1]))
        if st != ORC_OK:
            raise RuntimeError("oracle locate status %d" % st)
        return [int(v) for v in out[: nout.value]]

    def attach_ssa(self, samples, stride):
        """The row-sampled SSA of an index built elsewhere (for a BWT-only index: locate
        then walks LF over this BWT, fm_index.cpp:125-153, with these samples)."""
        s = np.ascontiguousarray(samples, np.uint64)
        lib().orc_attach_ssa(self._h, _u64(s) if len(s) else _u64(np.zeros(1, np.uint64)), len(s),
                             stride)

    def extract(self, pos, length):
        cap = max(1, min(length, self.n))
        out = np.zeros(cap, np.uint8)
        k = lib().orc_extract(self._h, pos, length, _u8(out))
        return bytes(out[:k])

    def count_batch(self, patterns=None, buf=None, offs=None, nthreads=1, faithful=False,
                    latencies=False):
        if patterns is not None:
            buf, offs = pack_patterns(patterns)
        buf = np.ascontiguousarray(buf, np.uint8)
        if len(buf) == 0:
            buf = np.zeros(1, np.uint8)
        offs = np.ascontiguousarray(offs, np.uint64)
        npat = len(offs) - 1
        out = np.zeros(max(npat, 1), np.uint64)
        lat = np.zeros(max(npat, 1), np.uint64) if latencies else None
        lib().orc_count_batch(self._h, _u8(buf), _u64(offs), npat, _u64(out), nthreads,
                              int(faithful), _u64(lat) if lat is not None else None)
        if latencies:
            return out[:npat], lat[:npat]
        return out[:npat]

    def locate_batch(self, patterns=None, buf=None, offs=None, limit=100000, nthreads=1,
                     faithful=False, cap=None):
        if patterns is not None:
            buf, offs = pack_patterns(patterns)
        buf = np.ascontiguousarray(buf, np.uint8)
        if len(buf) == 0:
            buf = np.zeros(1, np.uint8)
        offs = np.ascontiguousarray(offs, np.uint64)
        npat = len(offs) - 1
        if cap is None:
            cnt = self.count_batch(buf=buf, offs=offs, nthreads=nthreads)
            cap = int(np.minimum(cnt, limit).sum())
        out_offs = np.zeros(npat + 1, np.uint64)
        out_pos = np.zeros(max(cap, 1), np.uint64)
        st = lib().orc_locate_batch(self._h, _u8(buf), _u64(offs), npat, limit, _u64(out_offs),
                                    _u64(out_pos), cap, nthreads, int(faithful))
        if st == ORC_ERR_LF_OVERRUN:
            raise RuntimeError("locate: LF walk exceeded text length")
        if st != ORC_OK:
            raise RuntimeError("oracle locate_batch status %d" % st)
        return out_offs, out_pos[: int(out_offs[-1])]


# ---------------------------------------------------------------------------
def scan_count(text, pats, nloc=0, nthreads=8):
    """count() of every row of `pats` (npat x m bytes, one length) by scanning the text for
    its occurrences (orc_scan_count) — no index, so a full-size GPU index is checked against
    the text alone; equal to count() when the text ends in a unique smallest terminator
    (SURVEY.md §0.4).  nloc > 0: also the positions of the first nloc patterns, ascending
    (locate()'s positions in text order) -> (counts, offs[nloc+1], pos)."""
    t = as_u8(text)
    P = np.ascontiguousarray(pats, np.uint8)
    npat, m = P.shape
    counts = np.zeros(max(npat, 1), np.uint64)
    buf = P.reshape(-1) if P.size else np.zeros(1, np.uint8)
    tt = t if len(t) else np.zeros(1, np.uint8)
    if not nloc:
        st = lib().orc_scan_count(_u8(tt), len(t), _u8(buf), m, npat, _u64(counts), 0, None, None,
                                  0, nthreads)
        assert st == ORC_OK, st
        return counts[:npat]
    offs = np.zeros(nloc + 1, np.uint64)
    cap = 4 * nloc + 4096
    for _ in range(2):
        pos = np.zeros(cap, np.uint64)
        st = lib().orc_scan_count(_u8(tt), len(t), _u8(buf), m, npat, _u64(counts), nloc, _u64(offs),
                                  _u64(pos), cap, nthreads)
        if st == ORC_OK:
            return counts[:npat], offs, pos[: int(offs[-1])]
        cap = int(offs[-1])
    raise RuntimeError("orc_scan_count status %d" % st)


def check_suffix_array(text, sa, nthreads=8):
    """True iff `sa` is the suffix array of `text` in the reference's order (plain
    suffix order, a proper prefix first: src/core/sais.hpp:8-16): a permutation of
    0..n-1 whose consecutive suffixes strictly increase (orc_check_sa)."""
    t = as_u8(text)
    sa64 = np.ascontiguousarray(sa, np.uint64)
    if len(sa64) != len(t):
        return False
    if not len(t):
        return True
    return bool(lib().orc_check_sa(_u8(t), len(t), _u64(sa64), nthreads))


def sa_naive(text) -> np.ndarray:
    t = as_u8(text)
    out = np.zeros(max(len(t), 1), np.uint64)
    lib().orc_sa_naive(_u8(t if len(t) else np.zeros(1, np.uint8)), len(t), _u64(out))
    return out[: len(t)]


def sa_doubling(text) -> np.ndarray:
    t = as_u8(text)
    out = np.zeros(max(len(t), 1), np.uint64)
    lib().orc_sa_doubling(_u8(t if len(t) else np.zeros(1, np.uint8)), len(t), _u64(out))
    return out[: len(t)]


def gen_dna(seed: int, length: int) -> np.ndarray:
    """splitmix64, 32 bases per draw LSB-first, then '$'."""
    out = np.zeros(length + 1, np.uint8)
    lib().orc_gen_dna(seed, length, _u8(out))
    return out


def gen_rdna(seed: int, length: int) -> np.ndarray:
    """Repetitive DNA (cs_synth_text_device kind 2): copies of a 2^20-base seed sequence
    with ~0.75 % substitutions, then '$'."""
    out = np.zeros(length + 1, np.uint8)
    lib().orc_gen_rdna(seed, length, _u8(out))
    return out


def gen_bytes(seed: int, length: int) -> np.ndarray:
    out = np.zeros(length + 1, np.uint8)
    lib().orc_gen_bytes(seed, length, _u8(out))
    return out


def gen_patterns_text(text: np.ndarray, m: int, npat: int, seed: int = 4242) -> np.ndarray:
    """Q_text: npat x m matrix of substrings at x_k % (N - m)."""
    t = np.ascontiguousarray(text, np.uint8)
    out = np.zeros((max(npat, 1), m), np.uint8)
    lib().orc_gen_patterns_text(_u8(t), len(t), m, npat, seed, _u8(out))
    return out[:npat]


def gen_patterns_unif(kind: str, m: int, npat: int, seed: int = 4242) -> np.ndarray:
    """Q_unif as cs_synth_random_patterns_device: npat x m uniform random ACGT ("dna")
    or sigma=256-alphabet ("bytes") symbols from splitmix64."""
    out = np.zeros((max(npat, 1), m), np.uint8)
    lib().orc_gen_patterns_unif({"dna": 0, "bytes": 1}[kind], m, npat, seed, _u8(out))
    return out[:npat]


def gen_patterns_uniform(alphabet: bytes, m: int, npat: int, seed: int = 4243) -> np.ndarray:
    """Q_unif: uniform random patterns over `alphabet` (splitmix64 via numpy)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    a = np.frombuffer(alphabet, np.uint8)
    return a[rng.integers(0, len(a), size=(npat, m))]


# ---- the GENUINE reference (oracle/_ref/libcs_ref.so, built by `make -C oracle ref`
#      from the reference's own sources; test infrastructure / CPU baseline only) ----
_ref = None
REF_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref", "libcs_ref.so")


def ref_lib():
    """The reference shim (oracle/ref/ref_shim.cpp), or None when it is not built."""
    global _ref
    if _ref is None and os.path.exists(REF_LIB):
        R = C.CDLL(REF_LIB)
        R.ref_build_count_only.restype = C.c_void_p
        R.ref_build_count_only.argtypes = [C.POINTER(C.c_void_p), C.c_uint64, C.c_uint64, _u64p]
        R.ref_count_batch.restype = None
        R.ref_count_batch.argtypes = [C.c_void_p, _u8p, _u64p, C.c_uint64, C.c_int, _u64p, _u64p]
        R.ref_free.restype = None
        R.ref_free.argtypes = [C.c_void_p]
        R.ref_attach_locate.restype = None
        R.ref_attach_locate.argtypes = [C.c_void_p, _u8p, C.c_uint64, C.POINTER(C.c_uint32),
                                        C.c_uint64, C.c_uint32]
        R.ref_locate_batch.restype = None
        R.ref_locate_batch.argtypes = [C.c_void_p, _u8p, _u64p, C.c_uint64, C.c_uint64, C.c_int,
                                       C.c_uint64, C.POINTER(C.c_int64), _u64p, _u64p]
        if hasattr(R, "ref_csidx_open"):  # serialization.cpp in the shim (round 4)
            R.ref_csidx_open.restype = C.c_void_p
            R.ref_csidx_open.argtypes = [C.c_char_p, C.c_char_p, C.c_uint64]
            R.ref_csidx_close.restype = None
            R.ref_csidx_close.argtypes = [C.c_void_p]
            R.ref_csidx_header.restype = None
            R.ref_csidx_header.argtypes = [C.c_void_p, _u64p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
            R.ref_csidx_section.restype = C.c_void_p
            R.ref_csidx_section.argtypes = [C.c_void_p, C.c_int, _u64p, C.POINTER(C.c_uint32)]
        _ref = R
    return _ref


class RefCountIndex:
    """The reference's own FMIndex::count over this oracle index's wavelet levels
    (ref_build_count_only: genuine BitVector tables and count loop)."""

    def __init__(self, idx: "Index"):
        R = ref_lib()
        if R is None:
            raise FileNotFoundError(REF_LIB)
        ptrs = (C.c_void_p * 8)()
        nw = 0
        for l in range(8):
            ptrs[l], nw = idx.level(l).words_ptr()
        Cv = np.ascontiguousarray(idx.C(), np.uint64)
        self._h = R.ref_build_count_only(ptrs, nw, idx.n, _u64(Cv))
        self.n = idx.n

    def count_batch(self, buf, offs, nthreads=1, latencies=False):
        R = ref_lib()
        buf = np.ascontiguousarray(buf, np.uint8)
        if len(buf) == 0:
            buf = np.zeros(1, np.uint8)
        offs = np.ascontiguousarray(offs, np.uint64)
        npat = len(offs) - 1
        out = np.zeros(max(npat, 1), np.uint64)
        lat = np.zeros(max(npat, 1), np.uint64)
        R.ref_count_batch(self._h, _u8(buf), _u64(offs), npat, nthreads, _u64(out), _u64(lat))
        return (out[:npat], lat[:npat]) if latencies else out[:npat]

    def attach_locate(self, bwt, ssa, stride):
        """Give the index the members locate() reads (bwt_, ssa_): the reference's own
        FMIndex::locate (src/api/fm_index.cpp:107-157) then runs unmodified."""
        self._bwt = np.ascontiguousarray(bwt, np.uint8)
        self._ssa = np.ascontiguousarray(ssa, np.uint32)
        ref_lib().ref_attach_locate(self._h, _u8(self._bwt), len(self._bwt),
                                    self._ssa.ctypes.data_as(C.POINTER(C.c_uint32)),
                                    len(self._ssa), stride)
        del self._bwt, self._ssa  # copied into the reference's members

    def locate_batch(self, buf, offs, limit=100000, nthreads=1, cap=8):
        """-> (nout[q] (-1: the reference threw), positions[q, :cap], latency ns)."""
        R = ref_lib()
        buf = np.ascontiguousarray(buf, np.uint8)
        offs = np.ascontiguousarray(offs, np.uint64)
        npat = len(offs) - 1
        nout = np.zeros(max(npat, 1), np.int64)
        out = np.zeros((max(npat, 1), cap), np.uint64)
        lat = np.zeros(max(npat, 1), np.uint64)
        R.ref_locate_batch(self._h, _u8(buf), _u64(offs), npat, limit, nthreads, cap,
                           nout.ctypes.data_as(C.POINTER(C.c_int64)), _u64(out), _u64(lat))
        return nout[:npat], out[:npat], lat[:npat]

    def __del__(self):
        R = _ref
        if R is not None and getattr(self, "_h", None):
            R.ref_free(self._h)
            self._h = None


def ref_read_csidx(path):
    """A CSIDX file through the reference's own reader (cs::IndexReader, src/serialization/
    serialization.cpp:153-335, compiled into oracle/_ref/libcs_ref.so): {"text_len", "flags",
    "version", "text", "bwt", "C", "ssa", "stride"} as its getters return them (None for an
    absent section), or RuntimeError with the reader's exception text."""
    R = ref_lib()
    if R is None or not hasattr(R, "ref_csidx_open"):
        raise FileNotFoundError(REF_LIB)
    err = C.create_string_buffer(256)
    h = R.ref_csidx_open(path.encode(), err, 256)
    if not h:
        raise RuntimeError(err.value.decode())
    try:
        n, fl, ver = C.c_uint64(), C.c_uint32(), C.c_uint32()
        R.ref_csidx_header(h, C.byref(n), C.byref(fl), C.byref(ver))
        out = {"text_len": n.value, "flags": fl.value, "version": ver.value}
        for which, key, dt in ((0, "text", np.uint8), (1, "bwt", np.uint8), (2, "C", np.uint32),
                               (3, "ssa", np.uint32)):
            k, st = C.c_uint64(), C.c_uint32()
            ptr = R.ref_csidx_section(h, which, C.byref(k), C.byref(st))
            if not ptr:
                out[key] = None
                continue
            nb = k.value * np.dtype(dt).itemsize
            out[key] = np.frombuffer(C.string_at(ptr, nb), dt).copy() if nb else np.zeros(0, dt)
            if which == 3:
                out["stride"] = st.value
        return out
    finally:
        R.ref_csidx_close(h)
