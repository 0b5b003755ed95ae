#!/usr/bin/env python3
"""calibrate_cpu.py — TEST INFRASTRUCTURE: time the GENUINE reference's count()
(oracle/_ref/libcs_ref.so, built from /root/reference's sources by `make -C oracle
ref`) beside the C restatement's faithful count() (oracle/fm_oracle.c, faithful=1)
on the same index and the same Q_text 20-mers, single-threaded, at
n in {1e6, 8e6, 3.2e7} (the restatement must time within +-25 %
of the reference, so bench.py's cpu_baseline of kind "port" stands for the
reference's CPU path).  Runs in the build container only (the reference never
goes to the GPU box); writes profiles/r01/cpu_calibration.json.

    python oracle/calibrate_cpu.py [queries=16]
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import oracle as O  # noqa: E402


def ref_lib():
    R = C.CDLL(os.path.join(HERE, "_ref", "libcs_ref.so"))
    R.ref_build_from_sa.restype = C.c_void_p
    R.ref_build_from_sa.argtypes = [C.c_char_p, C.c_uint64, C.POINTER(C.c_uint32), C.c_uint32]
    R.ref_count.restype = C.c_uint64
    R.ref_count.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64]
    R.ref_free.argtypes = [C.c_void_p]
    return R


def main():
    Q = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    R = ref_lib()
    rows = []
    for n_bases in (999_999, 7_999_999, 31_999_999):
        t = O.gen_dna(42, n_bases)
        sa = O.sa_doubling(t.tobytes()).astype(np.uint32)
        h = R.ref_build_from_sa(t.tobytes(), len(t), sa.ctypes.data_as(C.POINTER(C.c_uint32)), 32)
        idx = O.Index(t.tobytes())
        pats = O.gen_patterns_text(t, 20, Q)
        t0 = time.perf_counter()
        rc = [int(R.ref_count(h, bytes(p), 20)) for p in pats]
        t_ref = time.perf_counter() - t0
        t0 = time.perf_counter()
        oc = [int(idx.count(bytes(p), faithful=True)) for p in pats]
        t_port = time.perf_counter() - t0
        R.ref_free(h)
        assert rc == oc, (n_bases, rc[:4], oc[:4])
        rows.append({"n": len(t), "queries": Q, "reference_s_per_query": t_ref / Q,
                     "port_s_per_query": t_port / Q, "port_over_reference": t_port / t_ref,
                     "counts_equal": True})
        print(json.dumps(rows[-1]), flush=True)
    out = {"what": "reference count() vs oracle faithful count(), 1 thread, Q_text 20-mers",
           "bar": "port within +-25 % of the reference (SURVEY.md §8(c))",
           "within_bar": all(0.75 <= r["port_over_reference"] <= 1.25 for r in rows),
           "host": os.uname().nodename, "rows": rows}
    path = os.path.join(ROOT, "profiles", "r01", "cpu_calibration.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
