#!/usr/bin/env python3
"""make_golden.py — regenerate tests/golden/*.json from the GENUINE reference.

Runs ONLY in the build container (needs /root/reference): `make -C oracle ref`
compiles oracle/_ref/ref_golden and oracle/_ref/libcs_ref.so from the reference's
own sources in place; this script feeds them inputs and records their outputs.
The committed JSON files are data (inputs + expected outputs); the GPU box and the
CPU test suite only read them.

Text inputs are stored literally (hex) when small, as a file name for the two data
files the reference ships (example.txt, sample.txt, copied here verbatim), or as a
generator spec {"gen": "dna"|"bytes", "seed", "len"} for the synthetic texts of
SURVEY.md §8(d) (regenerated bit-identically by oracle.gen_dna / gen_bytes).
"""
from __future__ import annotations

import ctypes as C
import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_golden")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libcs_ref.so")


def _hex(b: bytes) -> str:
    return bytes(b).hex()


def text_bytes(spec) -> bytes:
    if "hex" in spec:
        return bytes.fromhex(spec["hex"])
    if "file" in spec:
        with open(os.path.join(HERE, spec["file"]), "rb") as f:
            data = f.read()
        return data + bytes.fromhex(spec.get("append_hex", ""))
    if spec["gen"] == "dna":
        return O.gen_dna(spec["seed"], spec["len"]).tobytes()
    if spec["gen"] == "bytes":
        return O.gen_bytes(spec["seed"], spec["len"]).tobytes()
    raise ValueError(spec)


def run_ref_fm(text: bytes, patterns, stride: int, limit: int):
    with tempfile.TemporaryDirectory() as td:
        tp, pp = os.path.join(td, "t.bin"), os.path.join(td, "p.bin")
        with open(tp, "wb") as f:
            f.write(text)
        with open(pp, "wb") as f:
            f.write(struct.pack("<I", len(patterns)))
            for p in patterns:
                f.write(struct.pack("<I", len(p)) + p)
        out = subprocess.run([REF_BIN, "fm", tp, pp, str(stride), str(limit)], check=True,
                             capture_output=True, text=True).stdout.splitlines()
    counts, locs, extracts = [], [], []
    for line in out:
        tag, rest = line[0], line[2:]
        if tag == "C":
            counts.append(int(rest))
        elif tag == "L":
            v = [int(x) for x in rest.split()]
            locs.append({"pos": v[1:]})
        elif tag == "E":
            locs.append({"error": rest})
        elif tag == "X":
            v = [int(x) for x in rest.split()]
            extracts.append({"pos": v[0], "len": v[1], "hex": bytes(v[3:]).hex()})
    assert len(counts) == len(patterns) == len(locs)
    return counts, locs, extracts


def fm_case(name, text_spec, patterns, stride=32, limit=100000, note=""):
    text = text_bytes(text_spec)
    pats = [p.encode("latin-1") if isinstance(p, str) else bytes(p) for p in patterns]
    counts, locs, extracts = run_ref_fm(text, pats, stride, limit)
    return {"name": name, "note": note, "text": text_spec, "n": len(text), "ssa_stride": stride,
            "limit": limit, "patterns_hex": [_hex(p) for p in pats], "count": counts,
            "locate": locs, "extract": extracts}


def kat_cases():
    cases = []
    L = lambda s: {"hex": _hex(s.encode("latin-1") if isinstance(s, str) else s)}  # noqa: E731
    cases.append(fm_case("banana", L("banana$"),
                         ["banana", "ana", "na", "a", "b", "$", "x", "anana", "", "nan", "ban"],
                         note="tests/fm_search_tests.cpp:69-113, tests/simple_tests.cpp:6-13"))
    cases.append(fm_case("empty_text", L(""), ["", "x"], note="tests/fm_search_tests.cpp:56-60"))
    cases.append(fm_case("hello", L("hello$"), ["", "l", "ll", "hello$"],
                         note="tests/fm_search_tests.cpp:62-64"))
    cases.append(fm_case("no_match", L("abcdefg$"), ["xyz", "aaa", "gg", "g$", "abcdefg$"],
                         note="tests/fm_search_tests.cpp:115-128"))
    cases.append(fm_case("multiple_stride4", L("aabaabaa$"),
                         ["a", "aa", "aab", "b", "ba", "aba", "aabaabaa"], stride=4,
                         note="tests/fm_search_tests.cpp:130-152"))
    cases.append(fm_case("overlapping", L("abababab$"), ["ab", "aba", "abab", "b", "ba", "bab$"],
                         note="tests/fm_search_tests.cpp:154-173"))
    full = bytes(range(1, 256)) + b"$"
    cases.append(fm_case("full_alphabet", {"hex": _hex(full)},
                         [bytes([i]) for i in range(1, 256)] + [bytes([i, i + 1]) for i in range(1, 255, 17)],
                         note="tests/fm_search_tests.cpp:175-198; '$' occurs twice -> count 2 (reference output, assert at :191 contradicts it)"))
    long_text = ("The quick brown fox jumps over the lazy dog. The five boxing wizards jump quickly. "
                 "Pack my box with five dozen liquor jugs.$")
    cases.append(fm_case("long_text", L(long_text),
                         ["The", "the", "quick", "fox", "dog", "jump", "five", "box", "xyz", " ", ".",
                          "qu", "ing", "ck", "ox"], note="tests/fm_search_tests.cpp:237-251"))
    cases.append(fm_case("repeated", L("abcabcabcabc$"), ["abc", "ab", "bc", "ca", "abcabc", "a", "c"],
                         note="tests/fm_search_tests.cpp:253-261"))
    cases.append(fm_case("single_char", L("x$"), ["x", "y", "$", "x$"],
                         note="tests/fm_search_tests.cpp:263-278"))
    cases.append(fm_case("no_terminator_abab", L("abab"), ["ba", "ab", "a", "b", "aba", "bab"],
                         note="cyclic-rotation quirk, SURVEY.md §0.4"))
    cases.append(fm_case("example_cs_query", {"file": "example.txt"},
                         ["algorithm", "the", "quick", "FM-index", "compressed", "pattern matching",
                          "The", "$", "\n", "e", "data"], limit=100,
                         note="tools/query_cli.cpp semantics (no terminator, limit 100)"))
    cases.append(fm_case("example_build_index", {"file": "example.txt", "append_hex": "24"},
                         ["quick", "algorithm", "the", "$", "e"],
                         note="tools/build_index.cpp:63-66 appends '$'"))
    cases.append(fm_case("sample_cs_query", {"file": "sample.txt"}, ["banana", "ana", "band", "a", "n"],
                         limit=100, note="tools/query_cli.cpp on sample.txt"))
    rng = np.random.default_rng(7)
    for stride in (1, 2, 3, 5, 7, 16, 64):
        t = bytes(rng.choice(list(b"ACGT"), size=300).astype(np.uint8)) + b"$"
        pats = [t[i:i + m] for i, m in zip(rng.integers(0, 290, 25), rng.integers(1, 8, 25))]
        pats += [bytes(rng.choice(list(b"ACGT"), size=3).astype(np.uint8)) for _ in range(5)]
        cases.append(fm_case("dna300_stride%d" % stride, {"hex": _hex(t)}, pats, stride=stride,
                             note="SSA stride sweep"))
    for k, limit in ((0, 3), (1, 1), (2, 0)):
        t = bytes(rng.choice(list(b"ab"), size=200).astype(np.uint8)) + b"$"
        cases.append(fm_case("ab200_limit%d" % limit, {"hex": _hex(t)}, ["a", "ab", "ba", "aab", "bbb"],
                             limit=limit, note="locate limit truncation, row order"))
    t = bytes(rng.integers(0, 256, 400).astype(np.uint8))
    cases.append(fm_case("bytes400_noterm", {"hex": _hex(t)},
                         [t[i:i + 3] for i in range(0, 390, 37)] + [b"\x00", b"\xff", b"\x00\x00"],
                         note="random bytes incl. 0x00, no terminator"))
    return cases


def big_cases():
    cases = []
    dna = {"gen": "dna", "seed": 42, "len": 99999}
    t = text_bytes(dna)
    tn = np.frombuffer(t, np.uint8)
    q_text = O.gen_patterns_text(tn, 20, 1500, seed=4242)
    q_unif = O.gen_patterns_uniform(b"ACGT", 20, 500, seed=4243)
    short = [bytes(p) for p in O.gen_patterns_text(tn, 8, 200, seed=77)]
    pats = [bytes(p) for p in q_text] + [bytes(p) for p in q_unif] + short
    cases.append(fm_case("dna_100k", dna, pats, stride=32, limit=100000,
                         note="SURVEY §7 step 1: DNA n=1e5 incl. '$'; Q_text 20-mers (seed 4242), uniform 20-mers, 8-mers"))
    short2 = [bytes(p) for p in O.gen_patterns_text(tn, 4, 60, seed=78)]
    cases.append(fm_case("dna_100k_short_limit", dna, short2, stride=32, limit=40,
                         note="frequent 4-mers, limit 40 (row-order truncation)"))
    byt = {"gen": "bytes", "seed": 42, "len": 99999}
    tb = np.frombuffer(text_bytes(byt), np.uint8)
    pats = [bytes(p) for p in O.gen_patterns_text(tb, 8, 1500, seed=4242)]
    rng = np.random.default_rng(9)
    pats += [bytes(rng.integers(0, 256, 8).astype(np.uint8)) for _ in range(300)]
    pats += [bytes(p) for p in O.gen_patterns_text(tb, 2, 100, seed=79)]
    cases.append(fm_case("bytes_100k", byt, pats, stride=32, limit=100000,
                         note="sigma=256 n=1e5 incl. 0x00 terminator; 8-mers"))
    return cases


def bitvector_cases():
    out = []
    rng = np.random.default_rng(42)
    specs = [("zeros_100", np.zeros(100, np.uint8)), ("zeros_2048", np.zeros(2048, np.uint8)),
             ("ones_5000", np.ones(5000, np.uint8)), ("ones_2048", np.ones(2048, np.uint8)),
             ("one_bit_1", np.ones(1, np.uint8)), ("one_bit_0", np.zeros(1, np.uint8)),
             ("super_plus_1", np.concatenate([np.ones(2048, np.uint8), np.zeros(1, np.uint8)]))]
    for n in (500, 2048, 5000, 10000):
        specs.append(("random_%d" % n, rng.integers(0, 2, n).astype(np.uint8)))
    specs.append(("sparse_9000", (rng.random(9000) < 0.01).astype(np.uint8)))
    for name, bits in specs:
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "b.bin")
            bits.tofile(p)
            lines = subprocess.run([REF_BIN, "bv", p], check=True, capture_output=True,
                                   text=True).stdout.splitlines()
        _, n, ones = lines[0].split()
        r1 = [int(l.split()[0]) for l in lines[1:]]
        r0 = [int(l.split()[1]) for l in lines[1:]]
        out.append({"name": name, "bits_hex": np.packbits(bits, bitorder="little").tobytes().hex(),
                    "n": int(n), "count_ones": int(ones), "rank1": r1, "rank0": r0})
    return out


def wavelet_cases():
    out = []
    rng = np.random.default_rng(123)
    specs = [("banana", np.frombuffer(b"banana$", np.uint8), [ord(c) for c in "ban$x"]),
             ("single", np.frombuffer(b"x", np.uint8), [ord("x"), ord("y")]),
             ("all_z", np.full(1000, ord("z"), np.uint8), [ord("z"), ord("a")]),
             ("boundary", np.array([0, 255, 0, 255], np.uint8), [0, 255, 1]),
             ("alphabet_x2", np.concatenate([np.arange(256, dtype=np.uint8)] * 2), list(range(0, 256, 5)))]
    for n in (500, 2000, 5000):
        specs.append(("random_%d" % n, rng.integers(0, 256, n).astype(np.uint8),
                      [0, 1, 42, 100, 127, 128, 200, 255]))
    for name, seq, syms in specs:
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "w.bin")
            seq.tofile(p)
            lines = subprocess.run([REF_BIN, "wt", p, ",".join(map(str, syms))], check=True,
                                   capture_output=True, text=True).stdout.splitlines()
        ranks = {}
        acc = []
        for l in lines[1:]:
            v = l.split()
            if v[0] == "S":
                ranks[v[1]] = [int(x) for x in v[2:]]
            elif v[0] == "A":
                acc = [int(x) for x in v[1:]]
        out.append({"name": name, "seq_hex": seq.tobytes().hex(), "rank": ranks, "access": acc})
    return out


def ref_lib():
    R = C.CDLL(REF_SO)
    R.ref_build_from_sa.restype = C.c_void_p
    R.ref_build_from_sa.argtypes = [C.c_char_p, C.c_uint64, C.POINTER(C.c_uint32), C.c_uint32]
    R.ref_count.restype = C.c_uint64
    R.ref_count.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64]
    R.ref_locate.restype = C.c_int64
    R.ref_locate.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64, C.c_uint64,
                             C.POINTER(C.c_uint64), C.c_uint64]
    R.ref_free.argtypes = [C.c_void_p]
    return R


def mid_case():
    """n = 1e6 DNA through the genuine count/locate with members filled from the
    oracle's prefix-doubling SA (equal to build_sa_naive: tests pin it at small n)."""
    R = ref_lib()
    spec = {"gen": "dna", "seed": 42, "len": 999999}
    t = text_bytes(spec)
    sa = O.sa_doubling(t).astype(np.uint32)
    h = R.ref_build_from_sa(t, len(t), sa.ctypes.data_as(C.POINTER(C.c_uint32)), 32)
    tn = np.frombuffer(t, np.uint8)
    pats = [bytes(p) for p in O.gen_patterns_text(tn, 20, 400, seed=4242)]
    pats += [bytes(p) for p in O.gen_patterns_uniform(b"ACGT", 12, 100, seed=5)]
    counts, locs = [], []
    buf = (C.c_uint64 * 100000)()
    for p in pats:
        counts.append(int(R.ref_count(h, p, len(p))))
        k = R.ref_locate(h, p, len(p), 100000, buf, 100000)
        locs.append({"error": "exception"} if k < 0 else {"pos": list(buf[:k])})
    R.ref_free(h)
    return {"name": "dna_1m", "note": "genuine count/locate; members filled from a doubling SA "
            "(oracle/ref/ref_shim.cpp ref_build_from_sa)", "text": spec, "n": len(t),
            "ssa_stride": 32, "limit": 100000, "patterns_hex": [_hex(p) for p in pats],
            "count": counts, "locate": locs, "extract": []}


def main():
    if not os.path.exists(REF_BIN) or not os.path.exists(REF_SO):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    which = set(sys.argv[1:]) or {"kat", "big", "bv", "wt", "mid"}
    jobs = {"kat": ("fm_kat.json", kat_cases), "big": ("fm_100k.json", big_cases),
            "bv": ("bitvector.json", bitvector_cases), "wt": ("wavelet.json", wavelet_cases),
            "mid": ("fm_1m.json", lambda: [mid_case()])}
    for k in sorted(which):
        fname, fn = jobs[k]
        data = {"generator": "tests/golden/make_golden.py", "reference": "genuine (oracle/_ref)",
                "cases": fn()}
        with open(os.path.join(HERE, fname), "w") as f:
            json.dump(data, f, separators=(",", ":"))
        print("wrote", fname, os.path.getsize(os.path.join(HERE, fname)), "bytes")


if __name__ == "__main__":
    main()
