"""MI355X-native batched FM-index (Python mirror of the reference's cs::FMIndex).

Host-side mirror of src/api/fm_index.hpp:11-67 over the C ABI of
libcs_fmindex.so (include/cs_fmindex.h): same names, argument meaning and error
behaviour — RuntimeError with the reference's message where it throws
std::runtime_error.  Every query runs in the HIP kernels; there is no CPU
fallback: without the built library the import fails, and without a GPU every
call raises.

    idx = FMIndex.build_from_text(b"banana$", BuildParams())
    idx.count(b"ana")            # 2           (fm_index.cpp:79-101)
    idx.locate(b"ana")           # [3, 1]      (row order, fm_index.cpp:107-157)
    idx.count_batch([...])       # one launch for the whole batch
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libcs_fmindex.so")

CS_OK, CS_ERR_INVALID, CS_ERR_OOM, CS_ERR_HIP = 0, 1, 2, 3
CS_ERR_LF_OVERRUN, CS_ERR_SSA_RANGE, CS_ERR_CAPACITY, CS_ERR_UNSUPPORTED, CS_ERR_NO_DEVICE = 4, 5, 6, 7, 8

# query flags (include/cs_fmindex.h CS_Q_*): results unchanged, structures left out
Q_NO_PREFIX, Q_NO_CONTEXTS, Q_NO_FULL_SA, Q_NO_WALK_LINES, Q_NO_VERIFY, Q_LONG = 1, 2, 4, 8, 16, 32
Q_NO_LOC_RECORDS = 64
# tuning selectors (cs_fmindex.h CS_QT_*): equivalent kernels for tests and A/Bs, results
# unchanged; a handle's defaults come from the CS_FM_* environment when it is created
QT_BARRIER, QT_NO_ROUTE, QT_COUNT_U1, QT_COUNT_U4 = 1 << 8, 1 << 9, 1 << 10, 1 << 11
QT_LONG_LOADS8, QT_LONG_ROUND2, QT_LONG_BYTE_TEXT, QT_QCTX_UNSTAGED = 1 << 12, 1 << 13, 1 << 14, 1 << 15
QT_NO_ONEPASS, QT_ONEPASS_SA, QT_LOC_DEFER, QT_LOCATE_U1 = 1 << 16, 1 << 17, 1 << 18, 1 << 19
QT_WALK_ROWS, QT_WALK_PERSISTENT, QT_GENERAL_INLANE, QT_GENERAL_LIST_ALL = 1 << 20, 1 << 21, 1 << 22, 1 << 23
QT_MAP_LDS = 1 << 24

_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)
_vp = C.c_void_p


_opts_tls = threading.local()


def _options_text(options) -> str:
    if isinstance(options, dict):
        return " ".join(f"{k}={v}" for k, v in options.items())
    return str(options)


def _options_arg(options):
    """An explicit options string for cs_fm_build_with_options, or None."""
    return None if options is None else _options_text(options).encode()


def _set_thread_options(options):
    _check(lib().cs_fm_set_build_options(None if options is None else _options_text(options).encode()))


class build_options:
    """with build_options(ENGINE="wavelet", FULL_SA=0): every handle this thread constructs
    inside (build, create, open_directory, import) uses exactly these choices and reads no
    CS_FM_* environment variable (cs_fm_set_build_options); nested scopes replace, not merge."""

    def __init__(self, options=None, **kw):
        self.options = dict(options or {}, **kw)

    def __enter__(self):
        self.prev = getattr(_opts_tls, "current", None)
        _set_thread_options(self.options)
        _opts_tls.current = self.options
        return self

    def __exit__(self, *a):
        _set_thread_options(self.prev)
        _opts_tls.current = self.prev


def current_build_options():
    """The options of the innermost build_options() scope of this thread (None outside)."""
    return getattr(_opts_tls, "current", None)


class cs_build_params(C.Structure):
    _fields_ = [("S", C.c_uint32), ("s", C.c_uint32), ("ssa_stride", C.c_uint32), ("eps", C.c_double)]


class cs_count_out(C.Structure):
    _fields_ = [("d_counts", C.c_void_p), ("width", C.c_uint32), ("d_exc", C.c_void_p),
                ("exc_cap", C.c_uint64), ("d_exc_n", C.c_void_p)]


class cs_fm_info(C.Structure):
    _fields_ = [("n", C.c_uint64), ("ssa_stride", C.c_uint32), ("line_bits", C.c_uint32),
                ("lines_per_level", C.c_uint64), ("rank_bytes", C.c_uint64),
                ("ssa_bytes", C.c_uint64), ("active_levels", C.c_uint32 * 256), ("device", C.c_int),
                ("prefix_k", C.c_uint32), ("prefix_sigma", C.c_uint32), ("prefix_bytes", C.c_uint64),
                ("prefix_code", C.c_uint8 * 256), ("engine", C.c_uint32), ("line_bytes", C.c_uint32),
                ("levels", C.c_uint32), ("rare_rows", C.c_uint32), ("walk_marks", C.c_uint32),
                ("walk_bytes", C.c_uint64), ("context_q", C.c_uint32), ("position_stride", C.c_uint32),
                ("context_bytes", C.c_uint64), ("full_sa_bytes", C.c_uint64),
                ("record_bytes", C.c_uint32), ("text_in_hbm", C.c_uint32),
                ("packed_text_bytes", C.c_uint64), ("locate_record_bytes", C.c_uint64),
                ("locate_record_width", C.c_uint64), ("device_bytes", C.c_uint64)]


# Every entry point of include/cs_fmindex.h (and cs_fmindex_diag.h, cs_fmindex_replica.h, cs_synth.h)
# with its ctypes signature.
SIGNATURES = {
    "cs_default_build_params": (None, [C.POINTER(cs_build_params)]),
    "cs_fm_build_from_text": (C.c_int, [_u8p, C.c_uint64, C.POINTER(cs_build_params), C.c_int,
                                        C.POINTER(_vp)]),
    "cs_fm_build_from_device_text": (C.c_int, [_vp, C.c_uint64, C.POINTER(cs_build_params), C.c_int,
                                               C.POINTER(_vp)]),
    "cs_fm_build_with_options": (C.c_int, [_vp, C.c_uint64, C.c_int, C.POINTER(cs_build_params), C.c_char_p,
                                           C.c_int, C.POINTER(_vp)]),
    "cs_fm_set_build_options": (C.c_int, [C.c_char_p]),
    "cs_fm_open_directory": (C.c_int, [C.c_char_p, C.POINTER(_vp)]),
    "cs_fm_open_directory_on": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(_vp)]),
    "cs_fm_save_directory": (C.c_int, [_vp, C.c_char_p]),
    "cs_fm_open_csidx": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(_vp)]),
    "cs_fm_save_csidx": (C.c_int, [_vp, C.c_char_p]),
    "cs_csidx_check": (C.c_int, [C.c_char_p, _u64p, _u32p, C.POINTER(C.c_int)]),
    "cs_csidx_write": (C.c_int, [C.c_char_p, _u8p, C.c_uint64, _u32p, C.c_uint64, C.c_uint32, _u8p]),
    "cs_fm_destroy": (None, [_vp]),
    "cs_fm_get_info": (C.c_int, [_vp, C.POINTER(cs_fm_info)]),
    "cs_fm_last_error": (C.c_char_p, []),
    "cs_fm_count": (C.c_int, [_vp, C.c_char_p, C.c_uint64, _u64p]),
    "cs_fm_serve_start": (C.c_int, [_vp, C.c_uint32]),
    "cs_fm_serve_stop": (C.c_int, [_vp]),
    "cs_fm_locate": (C.c_int, [_vp, _u8p, C.c_uint64, C.c_uint64, _u64p, C.c_uint64, _u64p]),
    "cs_fm_extract": (C.c_int, [_vp, C.c_uint64, C.c_uint64, _u8p, _u64p]),
    "cs_fm_extract_batch": (C.c_int, [_vp, _u64p, _u64p, C.c_uint64, _u64p, _u8p, C.c_uint64,
                                      _u64p]),
    "cs_fm_count_batch": (C.c_int, [_vp, _u8p, _u64p, C.c_uint64, _u64p, _vp]),
    "cs_fm_locate_batch": (C.c_int, [_vp, _u8p, _u64p, C.c_uint64, C.c_uint64, _u64p, _u64p,
                                     C.c_uint64, _u64p, _vp]),
    "cs_fm_create": (C.c_int, [_u8p, C.c_uint64, _u32p, C.c_uint64, C.c_uint32, _u8p, C.c_int,
                               C.POINTER(_vp)]),
    "cs_fm_export_meta": (C.c_int, [_vp, C.c_char_p, C.c_uint64, _u64p, _u64p, _u32p]),
    "cs_fm_export_parts": (C.c_int, [_vp, C.POINTER(_vp), _vp]),
    "cs_fm_import": (C.c_int, [C.c_char_p, C.c_uint64, C.POINTER(_vp), C.c_uint32, C.c_int,
                               C.POINTER(_vp)]),
    "cs_fm_export_part_ptrs": (C.c_int, [_vp, C.POINTER(_vp), C.c_uint32]),
    "cs_fm_import_alloc": (C.c_int, [C.c_char_p, C.c_uint64, C.c_int, C.POINTER(_vp),
                                     C.POINTER(_vp), C.c_uint32]),
    "cs_fm_import_commit": (C.c_int, [_vp]),
    "cs_fm_extract_device": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint64, _vp, _vp]),
    "cs_fm_locate_record_hits_device": (C.c_int, [_vp, _vp, _vp, C.c_uint64, _vp, _vp]),
    "cs_fm_workspace_bytes": (C.c_uint64, [_vp, C.c_uint64]),
    "cs_fm_count_packed_device": (C.c_int, [_vp, _vp, C.c_uint32, C.c_uint64,
                                            C.POINTER(cs_count_out), C.c_uint32, _vp]),
    "cs_fm_locate_walk_steps_device": (C.c_int, [_vp, _vp, _vp, C.c_uint64, C.c_uint64, _vp,
                                                 C.c_uint32, _vp]),
    "cs_fm_locate_check": (C.c_int, [_vp, _vp]),
    "cs_fm_level_rank1": (C.c_int, [_vp, C.c_int, _u64p, C.c_uint64, _u64p]),
    "cs_fm_wt_rank": (C.c_int, [_vp, _u8p, _u64p, C.c_uint64, _u64p]),
    "cs_fm_wt_access": (C.c_int, [_vp, _u64p, C.c_uint64, _u8p]),
    "cs_fm_lf": (C.c_int, [_vp, _u64p, C.c_uint64, _u64p]),
    "cs_fm_get_C": (C.c_int, [_vp, _u64p]),
    "cs_fm_bwt_device": (C.c_int, [_vp, _vp, _vp]),
    "cs_fm_get_ssa": (C.c_int, [_vp, _u64p, C.c_uint64, _u64p]),
    "cs_sa_build": (C.c_int, [_u8p, C.c_uint64, _u32p, C.c_int]),
    "cs_counts_wire_bytes": (C.c_uint64, [C.c_uint64, C.c_uint64]),
    "cs_counts_pack_wire": (C.c_int, [_vp, C.c_uint64, C.c_uint64, _vp, _vp]),
    # include/cs_synth.h
    "cs_synth_text_device": (C.c_int, [C.c_int, C.c_uint64, C.c_uint64, _vp, _vp]),
    "cs_synth_patterns_device": (C.c_int, [_vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                           C.c_uint64, _vp, _vp, _vp]),
    "cs_synth_random_patterns_device": (C.c_int, [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64,
                                                   C.c_uint64, _vp, _vp, _vp]),
    # round 6: one count and one locate entry (flags + optional workspace), the two locate phases
    "cs_fm_count_device": (C.c_int, [_vp, _vp, _vp, C.c_uint64, C.c_uint64, C.POINTER(cs_count_out),
                                     C.c_uint32, _vp, C.c_uint64, _vp]),
    "cs_fm_locate_device": (C.c_int, [_vp, _vp, _vp, C.c_uint64, C.c_uint64, _vp, _vp, C.c_uint64,
                                      C.POINTER(C.c_uint64), C.c_uint32, _vp, C.c_uint64, _vp]),
    "cs_fm_locate_ranges_device": (C.c_int, [_vp, _vp, _vp, C.c_uint64, C.c_uint64, _vp, _vp,
                                             _u64p, C.c_uint32, _vp]),
    "cs_fm_locate_walk_device": (C.c_int, [_vp, _vp, _vp, C.c_uint64, C.c_uint64, _vp, C.c_uint32,
                                           C.c_int, _vp]),
    # include/cs_fmindex_diag.h (measurement twins; building blocks below)
    "cs_fm_count_bytes_device": (C.c_int, [_vp, _vp, _vp, C.c_uint64, _vp, C.c_uint32, _vp]),
}

_lib = None


def build(verbose: bool = False) -> str:
    """Compile libcs_fmindex.so for gfx950 in-tree (hipcc via the Makefile)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE, "-j8"], check=True,
                   stdout=None if verbose else subprocess.DEVNULL)
    return LIB_PATH


def lib():
    """Load the HIP library.  Fails loudly when it is missing: no fallback path."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libcs_fmindex.so not built: run `make -C %s` "
                              "(or __graft_entry__.build())" % _HERE)
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class FMIndexError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(msg)
        self.status = status


def _check(status: int):
    if status != CS_OK:
        raise FMIndexError(status, lib().cs_fm_last_error().decode("utf-8", "replace"))


def _bytes(x) -> bytes:
    if isinstance(x, str):
        return x.encode("latin-1")
    if isinstance(x, np.ndarray):
        return x.astype(np.uint8, copy=False).tobytes()
    return bytes(x)


def _u8(a: np.ndarray):
    return a.ctypes.data_as(_u8p)


def _u64(a: np.ndarray):
    return a.ctypes.data_as(_u64p)


def pack_patterns(patterns):
    """list of bytes-like -> (u8 concatenation, u64 offsets[n+1])."""
    pats = [_bytes(p) for p in patterns]
    offs = np.zeros(len(pats) + 1, np.uint64)
    if pats:
        offs[1:] = np.cumsum([len(p) for p in pats], dtype=np.uint64)
    buf = np.frombuffer(b"".join(pats) + b"\0", np.uint8).copy()
    return buf, offs


@dataclass
class BuildParams:
    """src/api/fm_index.hpp:11-14 (only ssa_stride shapes the index, as there)."""
    S: int = 512
    s: int = 64
    ssa_stride: int = 32
    eps: float = 1.0

    def _c(self):
        return cs_build_params(self.S, self.s, self.ssa_stride, self.eps)


class FMIndex:
    """cs::FMIndex (src/api/fm_index.hpp:17-67) backed by the MI355X engine."""

    def __init__(self, handle, n: int):
        self._h = handle
        self.n = n

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.cs_fm_destroy(h)
            self._h = None

    # -- construction (fm_index.hpp:19-20) --------------------------------
    @staticmethod
    def build_from_text(text, params: BuildParams | None = None, device: int | None = None,
                        options=None):
        """options: build choices (cs_fmindex_tuning.h cs_fm_build_with_options) as a dict
        {"ENGINE": "wavelet", "FULL_SA": 0} or a "NAME=VALUE ..." string; None takes the
        thread's build_options() scope, and outside one the CS_FM_* environment."""
        p = (params or BuildParams())._c()
        if device is None:
            device = int(os.environ.get("CS_FM_DEVICE", "0"))
        t = np.frombuffer(_bytes(text) + b"\0", np.uint8)
        n = len(t) - 1
        h = _vp()
        o = _options_arg(options)
        if o is None:
            _check(lib().cs_fm_build_from_text(_u8(t), n, C.byref(p), device, C.byref(h)))
        else:
            _check(lib().cs_fm_build_with_options(t.ctypes.data, n, 0, C.byref(p), o, device, C.byref(h)))
        return FMIndex(h, n)

    @staticmethod
    def build_from_device_text(d_text_ptr: int, n: int, params: BuildParams | None = None,
                               device: int = 0, options=None):
        p = (params or BuildParams())._c()
        h = _vp()
        o = _options_arg(options)
        if o is None:
            _check(lib().cs_fm_build_from_device_text(d_text_ptr, n, C.byref(p), device, C.byref(h)))
        else:
            _check(lib().cs_fm_build_with_options(d_text_ptr, n, 1, C.byref(p), o, device, C.byref(h)))
        return FMIndex(h, n)

    @staticmethod
    def create(bwt, ssa, ssa_stride: int = 32, text=None, device: int | None = None):
        """From host index arrays built elsewhere: the cyclic BWT and the row-sampled
        u32 SSA the reference's build_from_text leaves in bwt_ / ssa_
        (src/api/fm_index.cpp:49-66); `text` optional (kept for extract)."""
        if device is None:
            device = int(os.environ.get("CS_FM_DEVICE", "0"))
        b = np.frombuffer(_bytes(bwt) + b"\0", np.uint8)
        n = len(b) - 1
        sa = np.ascontiguousarray(ssa, np.uint32)
        if len(sa) == 0:
            sa = np.zeros(1, np.uint32)
        t = np.frombuffer(_bytes(text) + b"\0", np.uint8) if text is not None else None
        h = _vp()
        _check(lib().cs_fm_create(_u8(b), n, sa.ctypes.data_as(_u32p), len(ssa), ssa_stride,
                                  _u8(t) if t is not None else None, device, C.byref(h)))
        return FMIndex(h, n)

    # -- device image (replication across GPUs, shard.replicate_index) -----
    def export_meta(self):
        """-> (meta text bytes, [part sizes in bytes]) of the device image."""
        L = lib()
        ml, npart = C.c_uint64(), C.c_uint32()
        st = L.cs_fm_export_meta(self._h, None, 0, C.byref(ml), None, C.byref(npart))
        if st not in (CS_OK, CS_ERR_CAPACITY):
            _check(st)
        buf = C.create_string_buffer(ml.value)
        sizes = (C.c_uint64 * max(npart.value, 1))()
        _check(L.cs_fm_export_meta(self._h, buf, ml.value, C.byref(ml), sizes, C.byref(npart)))
        return buf.raw[: ml.value], [int(sizes[i]) for i in range(npart.value)]

    def export_parts(self, d_ptrs, stream=0):
        """Copy the image parts into device buffers d_ptrs (asynchronous on stream)."""
        arr = (_vp * len(d_ptrs))(*d_ptrs)
        _check(lib().cs_fm_export_parts(self._h, arr, stream or None))

    @staticmethod
    def import_image(meta: bytes, d_ptrs, device: int = 0):
        """An index on `device` from a meta text and device buffers holding the parts."""
        arr = (_vp * len(d_ptrs))(*d_ptrs)
        h = _vp()
        _check(lib().cs_fm_import(meta, len(meta), arr, len(d_ptrs), device, C.byref(h)))
        n = int(dict(l.split(" ", 1) for l in meta.decode().splitlines() if " " in l)["n"])
        return FMIndex(h, n)

    def export_part_ptrs(self, nparts: int):
        """Device addresses of the index's own image parts (read-only)."""
        arr = (_vp * max(nparts, 1))()
        _check(lib().cs_fm_export_part_ptrs(self._h, arr, nparts))
        return [int(arr[i] or 0) for i in range(nparts)]

    @staticmethod
    def import_alloc(meta: bytes, nparts: int, device: int = 0):
        """-> (index, [part addresses]): a handle with its parts allocated for the caller
        to fill (e.g. receive a broadcast into); call import_commit() afterwards."""
        arr = (_vp * max(nparts, 1))()
        h = _vp()
        _check(lib().cs_fm_import_alloc(meta, len(meta), device, C.byref(h), arr, nparts))
        n = int(dict(l.split(" ", 1) for l in meta.decode().splitlines() if " " in l)["n"])
        return FMIndex(h, n), [int(arr[i] or 0) for i in range(nparts)]

    def import_commit(self):
        _check(lib().cs_fm_import_commit(self._h))

    @staticmethod
    def open_directory(path: str, device: int | None = None):
        """Open an index written by save_directory (the reference's TODO,
        src/api/fm_index.hpp:20)."""
        if device is None:
            device = int(os.environ.get("CS_FM_DEVICE", "0"))
        h = _vp()
        _check(lib().cs_fm_open_directory_on(path.encode(), device, C.byref(h)))
        idx = FMIndex(h, 0)
        idx.n = idx.info().n
        return idx

    def save_directory(self, path: str):
        _check(lib().cs_fm_save_directory(self._h, path.encode()))

    @staticmethod
    def open_csidx(path: str, device: int | None = None):
        """Open a single-file index in the reference's CSIDX layout
        (src/serialization/serialization.hpp:1-83; BWT, SSA, C and text sections)."""
        if device is None:
            device = int(os.environ.get("CS_FM_DEVICE", "0"))
        h = _vp()
        _check(lib().cs_fm_open_csidx(path.encode(), device, C.byref(h)))
        idx = FMIndex(h, 0)
        idx.n = idx.info().n
        return idx

    def save_csidx(self, path: str):
        """Write the index as one CSIDX file (serialization.cpp:26-147's layout)."""
        _check(lib().cs_fm_save_csidx(self._h, path.encode()))


    # -- queries (fm_index.hpp:26-37) -------------------------------------
    def count(self, pattern) -> int:
        b = _bytes(pattern)
        out = C.c_uint64()
        _check(lib().cs_fm_count(self._h, b, len(b), C.byref(out)))
        return out.value

    def serve(self, on: bool = True, idle_us: int = 0):
        """Serving mode for single-pattern count(): a resident wave answers requests
        from a pinned mailbox instead of one kernel launch per call (cs_fm_serve_start;
        idle_us = idle exit, 0 = 10 ms).  serve(False) shuts it down."""
        if on:
            _check(lib().cs_fm_serve_start(self._h, idle_us))
        else:
            _check(lib().cs_fm_serve_stop(self._h))

    def locate(self, pattern, limit: int = 100000) -> list:
        offs, pos = self.locate_batch([pattern], limit)
        return [int(v) for v in pos]

    def extract(self, pos: int, length: int) -> bytes:
        cap = max(1, min(length, max(self.n - pos, 0)))
        out = np.zeros(cap, np.uint8)
        got = C.c_uint64()
        _check(lib().cs_fm_extract(self._h, pos, length, _u8(out), C.byref(got)))
        return out[: got.value].tobytes()

    def extract_batch(self, positions, lengths):
        """Device extract of many (pos, len) by LF inversion -> list of bytes."""
        p = np.ascontiguousarray(positions, np.uint64)
        l = np.ascontiguousarray(lengths, np.uint64)
        k = len(p)
        oo = np.zeros(k + 1, np.uint64)
        tot = C.c_uint64()
        st = lib().cs_fm_extract_batch(self._h, _u64(p), _u64(l), k, _u64(oo), None, 0,
                                       C.byref(tot))
        if st == CS_OK:
            return [b""] * k
        if st != CS_ERR_CAPACITY:
            _check(st)
        out = np.zeros(tot.value, np.uint8)
        _check(lib().cs_fm_extract_batch(self._h, _u64(p), _u64(l), k, _u64(oo), _u8(out),
                                         tot.value, C.byref(tot)))
        return [out[oo[q]:oo[q + 1]].tobytes() for q in range(k)]

    # -- batched ----------------------------------------------------------
    def count_batch(self, patterns=None, buf=None, offs=None) -> np.ndarray:
        if patterns is not None:
            buf, offs = pack_patterns(patterns)
        buf = np.ascontiguousarray(buf, np.uint8)
        if len(buf) == 0:
            buf = np.zeros(1, np.uint8)
        offs = np.ascontiguousarray(offs, np.uint64)
        npat = len(offs) - 1
        out = np.zeros(max(npat, 1), np.uint64)
        _check(lib().cs_fm_count_batch(self._h, _u8(buf), _u64(offs), npat, _u64(out), None))
        return out[:npat]

    def locate_batch(self, patterns=None, limit: int = 100000, buf=None, offs=None):
        """-> (out_offs[npat+1], positions) with positions of pattern q in row order at
        positions[out_offs[q]:out_offs[q+1]]."""
        if patterns is not None:
            buf, offs = pack_patterns(patterns)
        buf = np.ascontiguousarray(buf, np.uint8)
        if len(buf) == 0:
            buf = np.zeros(1, np.uint8)
        offs = np.ascontiguousarray(offs, np.uint64)
        npat = len(offs) - 1
        out_offs = np.zeros(npat + 1, np.uint64)
        total = C.c_uint64()
        st = lib().cs_fm_locate_batch(self._h, _u8(buf), _u64(offs), npat, limit, _u64(out_offs),
                                      None, 0, C.byref(total), None)
        if st == CS_OK:
            return out_offs, np.zeros(0, np.uint64)
        if st != CS_ERR_CAPACITY:
            _check(st)
        pos = np.zeros(total.value, np.uint64)
        _check(lib().cs_fm_locate_batch(self._h, _u8(buf), _u64(offs), npat, limit, _u64(out_offs),
                                        _u64(pos), total.value, C.byref(total), None))
        return out_offs, pos

    # -- device-resident batches (raw device pointers, e.g. torch data_ptr()) --
    def count_batch_device(self, d_pats: int, d_offs: int, npat: int, d_out: int, stream: int = 0):
        """count() of a device batch into uint64 counts (cs_fm_count_device, no flags)."""
        self.count_device_ws(d_pats, d_offs, npat, d_out, 0, 0, stream=stream)

    def count_fixed_device(self, d_pats: int, m: int, npat: int, d_out: int, stream: int = 0):
        """count of npat patterns of length m laid out back to back (no offsets array)."""
        self.count_device_ws(d_pats, None, npat, d_out, 0, 0, fixed_m=m, stream=stream)

    def extract_device(self, d_pos, d_len, d_out_offs, k, d_out, stream=0):
        """Batched extract with device buffers (d_out_offs = scan of clamped lengths)."""
        _check(lib().cs_fm_extract_device(self._h, d_pos, d_len, d_out_offs, k, d_out,
                                          stream or None))

    def count_device_ex(self, d_pats, d_offs, npat, d_out, width=8, flags=0, fixed_m=0,
                        d_exc=None, exc_cap=0, d_exc_n=None, stream=0):
        """count() of a device batch, general form (cs_fm_count_device without a workspace):
        d_offs or None for npat patterns of length fixed_m back to back; counts as uint64
        (width 8), uint32 (4) or uint8 with (index, count) pairs for counts >= 255 (1);
        flags Q_* leave structures out (same results)."""
        self.count_device_ws(d_pats, d_offs, npat, d_out, 0, 0, width, flags, fixed_m, d_exc, exc_cap,
                             d_exc_n, stream)

    def workspace_bytes(self, npat: int) -> int:
        """Device workspace for a count or one-call locate of up to npat patterns
        (cs_fm_workspace_bytes): zero-filled once by the caller, reused by its calls."""
        return int(lib().cs_fm_workspace_bytes(self._h, npat))

    def count_device_ws(self, d_pats, d_offs, npat, d_out, d_work, work_bytes, width=8, flags=0,
                        fixed_m=0, d_exc=None, exc_cap=0, d_exc_n=None, stream=0):
        """count() of a device batch (cs_fm_count_device) with the caller's workspace (no
        allocation inside the call; d_work 0: none)."""
        o = cs_count_out(d_out, width, d_exc, exc_cap, d_exc_n)
        _check(lib().cs_fm_count_device(self._h, d_pats, d_offs or None, fixed_m, npat, C.byref(o), flags,
                                        d_work or None, work_bytes, stream or None))

    def locate_device_ws(self, d_pats, d_offs, npat, limit, d_out_offs, d_out_pos, cap, d_work,
                         work_bytes, stream=0, flags=0):
        """locate_device with the caller's workspace (cs_fm_locate_device; d_work 0: none)."""
        total = C.c_uint64()
        st = lib().cs_fm_locate_device(self._h, d_pats, d_offs, npat, limit, d_out_offs,
                                       d_out_pos or None, cap, C.byref(total), flags,
                                       d_work or None, work_bytes, stream or None)
        if st == CS_ERR_CAPACITY:
            return total.value, False
        _check(st)
        return total.value, True

    def count_packed_device(self, d_packed, m, npat, d_out, width=8, flags=0, d_exc=None,
                            exc_cap=0, d_exc_n=None, stream=0):
        """count() of 2-bit packed DNA patterns (uint64 each, character i = "ACGT"[(x >> 2i)
        & 3], m <= 32): cs_fm_count_packed_device."""
        o = cs_count_out(d_out, width, d_exc, exc_cap, d_exc_n)
        _check(lib().cs_fm_count_packed_device(self._h, d_packed, m, npat, C.byref(o), flags,
                                               stream or None))

    def count_bytes_device(self, d_pats, d_offs, npat, d_out, stream=0, flags=0):
        """Per-query algorithmic HBM bytes of the search (roofline accounting)."""
        _check(lib().cs_fm_count_bytes_device(self._h, d_pats, d_offs, npat, d_out, flags,
                                              stream or None))

    def locate_record_hits_device(self, d_pats, d_offs, npat, d_hit, stream=0):
        """Per pattern 1 when the locate records answer it in one read (roofline accounting)."""
        _check(lib().cs_fm_locate_record_hits_device(self._h, d_pats, d_offs, npat, d_hit,
                                                     stream or None))

    def locate_ranges_device(self, d_pats, d_offs, npat, limit, d_sp, d_out_offs, stream=0,
                             flags=0) -> int:
        total = C.c_uint64()
        _check(lib().cs_fm_locate_ranges_device(self._h, d_pats, d_offs, npat, limit, d_sp,
                                                d_out_offs, C.byref(total), flags,
                                                stream or None))
        return total.value

    def locate_walk_device(self, d_sp, d_out_offs, npat, total, d_out_pos, stream=0, sync=True,
                           flags=0):
        """locate phase 2 (cs_fm_locate_walk_device); sync False: the overrun error goes to the
        next locate_check."""
        _check(lib().cs_fm_locate_walk_device(self._h, d_sp, d_out_offs, npat, total, d_out_pos, flags,
                                              1 if sync else 0, stream or None))

    def locate_device(self, d_pats, d_offs, npat, limit, d_out_offs, d_out_pos, cap, stream=0, flags=0):
        """locate of a batch in one call (cs_fm_locate_device, no workspace): offsets and, when
        they fit `cap`, positions -> (total, positions_written).  flags: Q_LONG sends every
        pattern to the long-pattern search."""
        return self.locate_device_ws(d_pats, d_offs, npat, limit, d_out_offs, d_out_pos, cap, 0, 0,
                                     stream, flags)

    def locate_walk_steps_device(self, d_sp, d_out_offs, npat, total, d_steps, stream=0, flags=0):
        """LF steps of each reported row's walk (measurement twin of the walk)."""
        _check(lib().cs_fm_locate_walk_steps_device(self._h, d_sp, d_out_offs, npat, total, d_steps,
                                                    flags, stream or None))

    def locate_check(self, stream=0):
        _check(lib().cs_fm_locate_check(self._h, stream or None))

    # -- building blocks / introspection ----------------------------------
    def info(self) -> cs_fm_info:
        inf = cs_fm_info()
        _check(lib().cs_fm_get_info(self._h, C.byref(inf)))
        return inf

    def C(self) -> np.ndarray:
        out = np.zeros(257, np.uint64)
        _check(lib().cs_fm_get_C(self._h, _u64(out)))
        return out

    def bwt_device(self, d_out: int, stream: int = 0):
        _check(lib().cs_fm_bwt_device(self._h, d_out, stream or None))

    def ssa(self) -> np.ndarray:
        ln = C.c_uint64()
        st = lib().cs_fm_get_ssa(self._h, None, 0, C.byref(ln))
        out = np.zeros(max(ln.value, 1), np.uint64)
        _check(lib().cs_fm_get_ssa(self._h, _u64(out), ln.value, C.byref(ln)))
        return out[: ln.value]

    def level_rank1(self, level: int, pos) -> np.ndarray:
        p = np.ascontiguousarray(pos, np.uint64)
        out = np.zeros(max(len(p), 1), np.uint64)
        _check(lib().cs_fm_level_rank1(self._h, level, _u64(p), len(p), _u64(out)))
        return out[: len(p)]

    def wt_rank(self, syms, pos) -> np.ndarray:
        s = np.ascontiguousarray(syms, np.uint8)
        p = np.ascontiguousarray(pos, np.uint64)
        out = np.zeros(max(len(p), 1), np.uint64)
        _check(lib().cs_fm_wt_rank(self._h, _u8(s), _u64(p), len(p), _u64(out)))
        return out[: len(p)]

    def wt_access(self, pos) -> np.ndarray:
        p = np.ascontiguousarray(pos, np.uint64)
        out = np.zeros(max(len(p), 1), np.uint8)
        _check(lib().cs_fm_wt_access(self._h, _u64(p), len(p), _u8(out)))
        return out[: len(p)]

    def lf(self, rows) -> np.ndarray:
        p = np.ascontiguousarray(rows, np.uint64)
        out = np.zeros(max(len(p), 1), np.uint64)
        _check(lib().cs_fm_lf(self._h, _u64(p), len(p), _u64(out)))
        return out[: len(p)]


def pack_dna(patterns) -> np.ndarray:
    """Equal-length ACGT patterns (m <= 32) -> one uint64 each, character i in bits 2i..2i+1
    (A=0, C=1, G=2, T=3): the input of count_packed_device."""
    pats = [_bytes(p) for p in patterns]
    lut = np.full(256, 255, np.uint8)
    for i, c in enumerate(b"ACGT"):
        lut[c] = i
    out = np.zeros(len(pats), np.uint64)
    if not pats:
        return out
    a = np.frombuffer(b"".join(pats), np.uint8).reshape(len(pats), -1)
    if a.shape[1] > 32:
        raise ValueError("packed DNA patterns hold at most 32 characters")
    d = lut[a]
    if (d == 255).any():
        raise ValueError("packed DNA patterns take A, C, G, T only")
    for i in range(a.shape[1]):
        out |= d[:, i].astype(np.uint64) << np.uint64(2 * i)
    return out


def synth_text_device(kind: str, seed: int, length: int, d_out: int, stream: int = 0):
    """SURVEY §8(d) text (kind 'dna' | 'bytes'), or 'rdna' (repetitive DNA: copies of a
    2^20-base seed with ~0.75 % substitutions); length+1 bytes incl. terminator."""
    k = {"dna": 0, "bytes": 1, "rdna": 2}[kind]
    _check(lib().cs_synth_text_device(k, seed, length, d_out, stream or None))


def synth_patterns_device(d_text: int, N: int, m: int, first: int, npat: int, seed: int,
                          d_pats: int, d_offs: int | None, stream: int = 0):
    """Q_text patterns [first, first+npat) of stream `seed`, fixed stride m."""
    _check(lib().cs_synth_patterns_device(d_text, N, m, first, npat, seed, d_pats, d_offs,
                                          stream or None))


def synth_random_patterns_device(kind: str, m: int, first: int, npat: int, seed: int,
                                 d_pats: int, d_offs: int | None, stream: int = 0):
    """Q_unif patterns [first, first+npat): uniform random symbols ("dna" / "bytes")."""
    k = {"dna": 0, "bytes": 1}[kind]
    _check(lib().cs_synth_random_patterns_device(k, m, first, npat, seed, d_pats, d_offs,
                                                 stream or None))


def counts_wire_bytes(npat: int, cap: int) -> int:
    """Size of the gather wire form of npat counts with cap overflow pairs."""
    return int(lib().cs_counts_wire_bytes(npat, cap))


def counts_pack_wire(d_counts: int, npat: int, cap: int, d_wire: int, stream: int = 0):
    """Pack a device uint64 count vector into its wire form (cs_counts_pack_wire)."""
    _check(lib().cs_counts_pack_wire(d_counts, npat, cap, d_wire, stream or None))


def sa_build(text, device: int = 0) -> np.ndarray:
    """Suffix array by the device builder (sais.hpp:8-16 order)."""
    t = np.frombuffer(_bytes(text) + b"\0", np.uint8)
    n = len(t) - 1
    out = np.zeros(max(n, 1), np.uint32)
    _check(lib().cs_sa_build(_u8(t), n, out.ctypes.data_as(_u32p), device))
    return out[:n]


def csidx_write(path: str, bwt, ssa, ssa_stride: int, text=None):
    """cs_csidx_write: a CSIDX file from host arrays (the reference's bwt_ / ssa_ / text_
    members) on the host, no device."""
    b = np.ascontiguousarray(np.frombuffer(bytes(bwt), np.uint8) if isinstance(bwt, (bytes, bytearray))
                             else bwt, np.uint8)
    s_ = np.ascontiguousarray(ssa, np.uint32)
    t = None
    if text is not None:
        t = np.ascontiguousarray(np.frombuffer(bytes(text), np.uint8) if isinstance(text, (bytes, bytearray))
                                 else text, np.uint8)
    _check(lib().cs_csidx_write(path.encode(), _u8(b) if len(b) else None, len(b),
                                s_.ctypes.data_as(_u32p) if len(s_) else None, len(s_), ssa_stride,
                                _u8(t) if t is not None and len(t) else None))


def csidx_check(path: str) -> dict:
    """Validate a CSIDX file on the CPU (no device): {"n", "ssa_stride", "has_text"};
    raises FMIndexError with the reason otherwise."""
    n = C.c_uint64()
    st = C.c_uint32()
    ht = C.c_int()
    _check(lib().cs_csidx_check(path.encode(), C.byref(n), C.byref(st), C.byref(ht)))
    return {"n": n.value, "ssa_stride": st.value, "has_text": bool(ht.value)}
