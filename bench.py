#!/usr/bin/env python3
"""bench.py — batched FM-index count() on MI355X (BASELINE.json metric).

Workload (default = BASELINE.json configs[3], "C4", the config the metric is
quoted on; it fits one GPU): 4 GB synthetic DNA text (n = 4e9 incl. the '$'
terminator, SURVEY.md §8(d): splitmix64 seed 42), Q_text 20-mers (substrings at
splitmix64(4242) positions).  One step = one batched count() launch over a batch
of --batch patterns per GPU, inputs resident in HBM, uint64 counts (the
reference's FMIndex::count return type).  Multi-GPU: one process per GPU, index
replicated (built per GPU), query stream sharded in contiguous ranges (weak
scaling: --batch per GPU); every step's counts are gathered to rank 0 over RCCL
 in their exact 1-B wire form (cs_counts_pack_wire), the gather of
step k overlapped with the count of step k+1; the timed region closes after the
last gather.

Output: ONE compact JSON line on stdout (<= 4 KB, compact_line(): the contract's fields, the
count kernel's roofline, cpu_baseline, p50 and a locate summary), and the full result below
— every leg — in the --legs-out file (default gpurun_out/bench_full_n<N>_<time>.json) and on
stderr.

Fields of the full result:
  roofline     the count kernel against HBM: achieved = algorithmic bytes per
               launch / mean kernel time (HIP events on the launch stream).
               Algorithmic bytes = the random reads the search needs (prefix-table
               entry or context record, one 32-B line per rank step, the 32-B context
               sector(s); counted per query by cs_fm_count_bytes_device) + the stream
               every launch moves (patterns, offsets, counts).  traffic = HBM bytes per
               launch from the committed rocprofv3 PMC summary for this workload.
  legs         (N=1) the same batch through the other query forms and structures,
               each with its own roofline: the reference's plain backward-search loop
               (CS_Q_NO_CONTEXTS: table + rank steps; CS_Q_NO_PREFIX|NO_CONTEXTS: every
               step through the occurrence lines), longer patterns (m = 32, 64),
               uint32 counts, 2-bit packed patterns, the reference's own 8-level
               binary wavelet matrix (its table + steps and its whole LF loop), and
               locate with the full SA, the reference's row-sampled SSA walk (stride
               32) and the walk lines.
  cpu_baseline the reference's own FMIndex::count (oracle/_ref/libcs_ref.so, built
               from its sources; kind "reference"), else the oracle's
               reference-faithful count() (kind "port"; O(n) count_ones scans, as
               src/core/bitvector.cpp:168-170), on a bounded sample of the same
               batch, rank 0, N=1 only, on the process's CPU share; cpu_locate: the
               reference's FMIndex::locate the same way.
  p50_us       median end-to-end latency of single-pattern cs::FMIndex::count() calls
               through the C++ facade (host pattern in, count out), as
               tools/benchmark.cpp:154-166, with the index in serving mode (a resident
               wave answers from a pinned mailbox); p50_launch_us: the same calls with
               one kernel launch each.
--only LEG runs one leg and nothing else (the rocprofv3 passes of
profiles/profile_legs.sh); --legs chooses the legs of a full run.
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from __graft_entry__ import _load_pkg  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# measured random-read ceiling of MI355X: profiles/microbench/gather_bench.hip, 8..32-B
# random reads over a 4 GB table at 49-52 G accesses/s (profiles/r01/gather_bench*.txt)
RANDOM_CEIL = 5.0e10
# the same microbenchmark by table size and read width (profiles/r01, r02, r04 gather_bench_*g
# .txt, `indep`, grid 8192): random reads are dearer over larger tables (address translation
# reach), so a leg's accesses are set against the ceiling of the structure they hit — the
# record table (16 B) for the headline, the 2-GB occurrence lines (32-B lines) for the
# reference's loop
RANDOM_CEIL_BY_GB = {16: ((1, 54.3e9), (2, 53.2e9), (4, 51.9e9), (17, 48.0e9), (32, 47.2e9), (34, 48.6e9),
                          (69, 47.1e9)),
                     32: ((1, 54.0e9), (2, 53.5e9), (4, 48.6e9), (17, 39.1e9), (32, 38.5e9), (34, 38.4e9),
                          (69, 38.0e9))}


HOT_TABLE_BYTES = 1 << 30  # the smallest table measured: the best random-read rate
DRAM_ACCESS = 64.0  # HBM bytes per random read request (profiles/summarize_legs.py)


def random_ceiling(table_bytes, width):
    """The measured random-read rate for `width`-byte reads over a table of `table_bytes`
    (nearest measured size below, else the smallest); None = RANDOM_CEIL."""
    pts = RANDOM_CEIL_BY_GB.get(16 if width and width <= 16 else 32)
    if not table_bytes or not pts:
        return RANDOM_CEIL
    gb = table_bytes / 1e9
    below = [r for g, r in pts if g <= gb * 1.05]
    return below[-1] if below else pts[0][1]
# (round 5: the "access-mix ceiling" of rounds 2-4 — gather_bench k_mixed, 33.5 G accesses/s
# — is gone: legs beside it ran up to 1.6x above it, so it bounded nothing, VERDICT r04 weak
# item 6)
# The MI355X's Infinity Cache (MALL): a leg whose random reads hit a table that fits it is
# cache-bound, not HBM-bound (MI355X_MICROARCH.md: 256 MiB)
MALL_BYTES = 256 << 20
PMC_LEGS = os.path.join(ROOT, "profiles", "pmc_legs.json")
sys.path.insert(0, os.path.join(ROOT, "profiles"))
from srchash import kernel_src_hash  # noqa: E402  (the key of a PMC profile)
SRC_HASH = kernel_src_hash()

# legs by index: the headline index (occurrence lines + contexts + records + full SA),
# the reference's binary wavelet matrix, the occurrence engine with walk lines
LEGS_MAIN = ["count_100m", "count_streams", "count_u32", "count_packed", "count_table_steps", "count_lf_loop", "count_m32",
             "count_m64", "count_m64_steps", "count_m150", "count_m150_staged", "count_m64_long", "count_m150_long",
             "count_fixed", "count_unif", "locate", "locate_one", "locate_ssa_rows",
             "locate_m64", "locate_m150", "locate_m64_steps", "count_stream", "count_stream_packed",
             "count_stream_packed_u8", "host_batch",
             "extract"]
LEGS_WM = ["wm_count", "wm_lf_loop", "wm_locate_ssa"]
LEGS_WALK = ["locate_ssa"]
# the learned occurrence lines (the reference's learned occ, as int16
# residuals against a per-superblock linear model): the headline and the whole LF loop
LEGS_LEARNED = ["learned_count", "learned_lf_loop"]
# repetitive DNA of the same size (cs_synth_text_device kind 2): heavy-tailed ranges
LEGS_RDNA = ["count_rdna", "locate_rdna"]
# the HBM footprint / throughput trade-off: the same text indexed with the optional
# structures added one at a time
LEGS_FOOT = ["footprint", "budget"]
# CS_FM_HBM_BUDGET values of the budget leg, as fractions of the default index's footprint
BUDGET_FRACS = (0.3, 0.6)
ALL_LEGS = LEGS_MAIN + LEGS_WM + LEGS_WALK + LEGS_LEARNED + LEGS_RDNA + LEGS_FOOT

# footprint ladder rungs: (name, what the rung adds, build switches)
_OFF = {"CS_FM_PREFIX_K": "0", "CS_FM_LCTX": "0", "CS_FM_CTX_RECORDS": "0", "CS_FM_FULL_SA": "0",
        "CS_FM_DEVICE_TEXT": "0", "CS_FM_WALK": "0"}
FOOT_RUNGS = [
    ("minimal", "occurrence lines, row-sampled SSA and inverse-SA samples at the SSA stride: "
     "the reference's members (bwt_ as lines, ssa_)", dict(_OFF, CS_FM_PSTRIDE="32")),
    ("walk_lines", "+ walk lines (locate: LF + mark + sample index in one line)",
     dict(_OFF, CS_FM_WALK="1")),
    ("prefix_table", "+ k-mer prefix table (count: the first k steps in one read)",
     dict(_OFF, CS_FM_WALK="1", CS_FM_PREFIX_K="")),
    ("left_contexts", "+ left contexts (count: the last <= 7 steps in one read)",
     dict(_OFF, CS_FM_WALK="1", CS_FM_PREFIX_K="", CS_FM_LCTX="")),
    ("context_records", "+ context records (count: one read)",
     dict(_OFF, CS_FM_WALK="1", CS_FM_PREFIX_K="", CS_FM_LCTX="", CS_FM_CTX_RECORDS="")),
    ("full_sa_text", "+ full suffix array and the text (locate one SA read after the record, "
     "extract a copy)", {"CS_FM_LOC_RECORDS": "0"}),
    ("full", "+ locate records (the default build, round 4: a Q_text 20-mer's position in one "
     "16-B read)", {}),
]


class LegGuard:
    """A failing leg (or the CPU baseline / p50 block) is reported in the JSON line's
    "leg_errors" instead of losing the whole line."""

    def __init__(self, errs, name):
        self.errs, self.name = errs, name

    def __enter__(self):
        return self

    def __exit__(self, et, ev, tb):
        if et is None or issubclass(et, KeyboardInterrupt):
            return False
        import traceback
        traceback.print_exception(et, ev, tb, file=sys.stderr)
        self.errs[self.name] = "%s: %s" % (et.__name__, ev)
        try:
            torch.cuda.synchronize()
        except Exception:
            pass
        return True


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


# the stdout line must survive a reader that keeps only the last few KB of the run's output
# (round 3's 46-KB line with every leg inside was cut to its tail): the headline fields below,
# the full result (every leg) in the --legs-out file and on stderr
LINE_MAX = 4096
_ROOF_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "alg_bytes_per_launch",
              "kernel_ms_median", "kernel_ms_mean", "frac_of_random_access_ceiling", "traffic_frac")
_CPU_KEYS = ("value", "unit", "cores", "kind", "cores_used", "host_cores", "matches_gpu", "p50_us",
             "per_core_value")
_CFG_KEYS = ("workload", "batch_per_gpu", "global_batch", "m", "ssa_stride", "parallelism", "index")


def _sig(x, d=4):
    """Round floats to d significant digits (the line's numbers, not its precision claims)."""
    if isinstance(x, float):
        return float("%.*g" % (d, x))
    if isinstance(x, dict):
        return {k: _sig(v, d) for k, v in x.items()}
    if isinstance(x, list):
        return [_sig(v, d) for v in x]
    return x


def compact_line(res, legs_file=None):
    """The one stdout JSON line: the headline of `res` (bench.py's full result) in at most
    LINE_MAX bytes.  Kept: the contract's fields, the count kernel's roofline, the CPU
    baseline, p50 and a two-number locate summary; the legs stay in the full result.  Fields
    are dropped from the end of an optional list until the line fits."""
    if "only" in res:  # profiling passes (--only): the leg object is the whole point
        return json.dumps(res)
    out = {k: res[k] for k in ("metric", "value", "unit", "n_gpus", "ranks_seen", "steps", "warmup",
                               "ms_per_step", "higher_is_better", "scaling", "vs_baseline", "dtype",
                               "data") if k in res}
    if "value" in out:
        out["value"] = float("%.6g" % out["value"])
    if "config" in res:
        out["config"] = {k: res["config"][k] for k in _CFG_KEYS if k in res["config"]}
    rf = res.get("roofline")
    if rf:
        out["roofline"] = _sig({k: rf.get(k) for k in _ROOF_KEYS})
    cb = res.get("cpu_baseline")
    if cb:
        out["cpu_baseline"] = _sig({k: cb.get(k) for k in _CPU_KEYS if k in cb})
        out["cpu_baseline"]["sample"] = str(cb.get("sample", ""))[:160]
    for k in ("p50_us", "p99_us", "p50_launch_us", "p99_launch_us"):
        if k in res:
            out[k] = _sig(res[k])
    loc = res.get("locate")
    if loc:
        rl = loc.get("roofline") or loc.get("walk_roofline") or {}
        out["locate"] = _sig({"patterns_per_s": loc.get("patterns_per_s"), "frac": rl.get("frac")})
    # the index's whole HBM footprint (every allocation of the handle, cs_fm_info.device_bytes)
    # and the rate at BASELINE configs[3]'s whole 100 M batch in one call
    if res.get("index_hbm_bytes"):
        out["index_hbm_bytes"] = res["index_hbm_bytes"]
    c100 = (res.get("legs") or {}).get("count_100m")
    if isinstance(c100, dict) and c100.get("patterns_per_s"):
        out["count_100m_patterns_per_s"] = _sig(c100["patterns_per_s"])
    opt = []  # optional, dropped last-first while the line is too long
    if "gather_verified" in res:
        out["gather_verified"] = res["gather_verified"]
    if res.get("leg_errors"):
        out["leg_errors"] = sorted(res["leg_errors"])[:8]
        opt.append("leg_errors")
    if legs_file:
        out["legs_file"] = legs_file
        opt.append("legs_file")
    if "found_frac" in res:
        out["found_frac"] = _sig(res["found_frac"])
        opt.append("found_frac")
    if res.get("config", {}).get("engine"):
        out["config"]["engine"] = res["config"]["engine"]
        opt.append(("config", "engine"))
    line = json.dumps(out)
    while len(line.encode()) > LINE_MAX and opt:
        k = opt.pop()
        if isinstance(k, tuple):
            out[k[0]].pop(k[1], None)
        else:
            out.pop(k, None)
        line = json.dumps(out)
    if len(line.encode()) > LINE_MAX:  # never expected: the kept fields are bounded
        out.pop("cpu_baseline", None)
        out["config"] = {"workload": str(out.get("config", {}).get("workload", ""))[:200]}
        line = json.dumps(out)
    return line


def pmc_traffic(wl, leg, kern_s):
    """HBM bytes per launch of `leg` on workload `wl` from the committed PMC summaries
    (profiles/pmc_legs.json), -> {"traffic", "traffic_stale", "traffic_profile"}.  A profile
    describes the code that ran only if it was taken from the same kernel sources: each entry
    carries the source hash of the tree it was profiled from (profiles/srchash.py), and the
    traffic is attached only when it equals this tree's hash — else traffic is null and
    traffic_stale true (round 6, VERDICT r05 item 4: rounds 4-5 admitted a profile whose
    kernel time was within +-15 % of this run's, and a similar time is no evidence of similar
    traffic).  `kern_s` (this run's kernel time) is reported beside the profiled time."""
    e = json.load(open(PMC_LEGS)).get("%s|%s" % (wl, leg)) if os.path.exists(PMC_LEGS) else None
    if not e:
        return {"traffic": None, "traffic_stale": None, "traffic_profile": None}
    prof_s = (e.get("kernel_median_ns_profiled") or e.get("kernel_mean_ns_profiled", 0)) / 1e9
    fresh = bool(e.get("src_hash")) and e.get("src_hash") == SRC_HASH
    return {"traffic": e.get("hbm_bytes_per_launch") if fresh else None, "traffic_stale": not fresh,
            "traffic_profile": {"tag": e.get("tag"), "kernel": e.get("kernel"),
                                "kernel_ms_profiled": prof_s * 1e3,
                                "kernel_ms_this_run": kern_s * 1e3 if kern_s else None,
                                "src_hash": e.get("src_hash"), "src_hash_this_run": SRC_HASH,
                                "l2_hit_rate": e.get("l2_hit_rate")}}


def time_launches(launch, steps, warmup, stream):
    """warmup + timed launches -> (wall s per launch, kernel s per launch (HIP events on
    the launch stream), min kernel ms)."""
    for _ in range(warmup):
        launch()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    t0 = time.perf_counter()
    for k in range(steps):
        evs[k][0].record(stream)
        launch()
        evs[k][1].record(stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    ms = [a.elapsed_time(b) for a, b in evs]
    return wall, statistics.mean(ms) / 1e3, min(ms)


class Workload:
    """Device batch of B patterns of length m (Q_text or Q_unif) + its accounting."""

    def __init__(self, pkg, text, N, m, lo, B, kind, queries, dev, sh):
        self.m, self.B = m, B
        self.pats = torch.empty(B * m, dtype=torch.uint8, device=dev)
        self.offs = torch.empty(B + 1, dtype=torch.int64, device=dev)
        if queries == "text":
            pkg.synth_patterns_device(text.data_ptr(), N, m, lo, B, 4242, self.pats.data_ptr(),
                                      self.offs.data_ptr(), sh)
        else:  # SURVEY §8(d) secondary batch Q_unif
            pkg.synth_random_patterns_device(kind, m, lo, B, 4242, self.pats.data_ptr(),
                                             self.offs.data_ptr(), sh)

    def accounting(self, idx, info, flags, sh, dev):
        """-> (random algorithmic bytes per launch, random accesses per launch, table hit
        fraction).  Random bytes from the engine's measurement twin
        (cs_fm_count_bytes_device): per backward-search step the distinct lines its rank
        pair (sp, ep) needs times the line size, the prefix-table entry / context
        record, the context sector(s)."""
        B, m = self.B, self.m
        qb = torch.empty(B, dtype=torch.int64, device=dev)
        idx.count_bytes_device(self.pats.data_ptr(), self.offs.data_ptr(), B, qb.data_ptr(), sh,
                               flags=flags)
        rnd = int(qb.sum().item())
        del qb
        K = 0 if flags & 1 else info.prefix_k
        frac = 0.0
        if K and m >= K:
            # (in chunks of 4 M patterns: the int64 temporaries of a 100 M batch would take
            # 28 GB beside C5's 237-GB index)
            code = torch.tensor(list(info.prefix_code), dtype=torch.int64, device=dev)
            P = self.pats.view(B, m)
            hit = 0
            for a0 in range(0, B, 1 << 22):
                P2 = P[a0:a0 + (1 << 22), m - K:].long()
                hit += int((code[P2] != 255).all(dim=1).sum().item())
                del P2
            frac = hit / B
        eb = info.prefix_bytes // (info.prefix_sigma ** K) if K else 0
        hits = int(round(B * frac)) if K else 0
        acc = (rnd - eb * hits) / info.line_bytes + hits
        return rnd, acc, frac


def dram_basis(alg, stream_read, accesses, pmc):
    """What the roofline fractions are taken on: with a fresh PMC
    profile of the leg, the bytes are min(algorithmic, measured HBM traffic) — cache hits
    (the first backward-search steps from C[] share lines across patterns) are not HBM
    reads — and the random accesses likewise min(algorithmic, the DRAM's): the traffic is
    the stream plus one 64-B DRAM request per random read (profiles/summarize_legs.py
    DRAM_ACCESS: the count kernels' requests are all 64 B, TCC_EA0_RDREQ_32B_sum = 0), so
    requests = (traffic - stream) / 64.  Without a fresh profile, the algorithmic figures.
    -> (bytes, random accesses, basis)."""
    tr = pmc.get("traffic")
    if tr:
        return min(alg, tr), min(accesses, max(0.0, (tr - (stream_read or 0)) / DRAM_ACCESS)), "pmc"
    return alg, accesses, "algorithmic"


def ceiling_frac(rate, ceil, table_bytes):
    """(bound, fraction of the random-read ceiling) of a leg reading `rate` random accesses/s
    from a table of `table_bytes`: "mall" (no fraction) when the table fits the 256-MiB
    Infinity Cache, "cache" (no fraction) when the rate passes the HBM ceiling — reads served
    partly by the L2 / MALL — else "hbm" and rate / ceiling (<= 1)."""
    if table_bytes and table_bytes <= MALL_BYTES:
        return "mall", None
    f = rate / ceil
    return ("cache", None) if f > 1.0 else ("hbm", f)


def roofline(alg_random, alg_stream, accesses, kern_s, B, pmc, stream_read=None, table=None):
    """pmc: pmc_traffic()'s dict (traffic + whether its profile matches this kernel);
    table: (bytes, read width) of the structure the random reads hit."""
    alg = alg_random + alg_stream
    fb, acc, basis = dram_basis(alg, stream_read, accesses, pmc)
    ceil = random_ceiling(*table) if table else RANDOM_CEIL
    achieved = fb / kern_s / 1e9
    # the measured random-read ceiling binds a leg whose reads go to HBM: a table that fits the
    # 256-MiB MALL is "mall"-bound (C2's occurrence lines), and a leg whose reads run above the
    # HBM ceiling is served partly by the L2 / MALL (the first backward-search steps from C[]
    # share lines across patterns: FETCH_SIZE counts those hits too) — "cache", no fraction
    bound, frac_c = ceiling_frac(acc / kern_s, ceil, table[0] if table else None)
    return {"bound": bound, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, **pmc, "basis": basis,
            "alg_bytes_per_launch": alg, "alg_random_bytes_per_launch": alg_random,
            "alg_stream_bytes_per_launch": alg_stream, "alg_bytes_per_query": alg / B,
            "alg_GBs": alg / kern_s / 1e9,
            "stream_read_bytes_per_launch": stream_read,
            "alg_random_accesses_per_launch": accesses,
            "random_accesses_per_launch": acc,
            "random_accesses_per_query": acc / B,
            "random_accesses_per_s": acc / kern_s,
            "random_access_ceiling_per_s": ceil,
            "random_access_table_bytes": table[0] if table else None,
            "frac_of_random_access_ceiling": frac_c,
            # the HBM's own load: the measured traffic (PMC, 64-B requests) per second
            # against the peak — the random-read regime moves 64 B per 16-B record
            "traffic_frac": (pmc.get("traffic") or 0) / kern_s / 1e9 / HBM_PEAK_GBS or None}


def count_leg(name, what, idx, info, wl_key, W, launch, flags, stream_bytes, steps, warmup,
              stream, sh, dev, ref_counts, read_counts, stream_read=None):
    """Time one count form over workload W; check its counts against ref_counts.
    stream_bytes: the bytes every launch streams (patterns, offsets, counts written);
    stream_read: the read part of them (default: the patterns and their offsets)."""
    if stream_read is None:
        stream_read = W.B * W.m + (W.B + 1) * 8
    wall, kern_s, kmin = time_launches(launch, steps, warmup, stream)
    rnd, acc, frac = W.accounting(idx, info, flags, sh, dev)
    # the structure most random reads hit: the rank lines when the search steps (the whole
    # loop, no contexts, no verification), else the table of context records / entries
    # — except that the rank steps' lines are not spread over the table: every pattern's
    # first steps from C[] (or from a table range) read the same few lines, which stay in
    # the L2 / the 256-MB MALL (FETCH_SIZE counts MALL hits as fetches), so those legs are
    # set against the best measured random rate (a 1-GB table) rather than the table's size
    steps_mostly = flags & (1 | 2 | 16)
    table = ((HOT_TABLE_BYTES, info.line_bytes) if steps_mostly
             else (info.rank_bytes, info.line_bytes) if not info.prefix_bytes
             else (info.prefix_bytes, info.record_bytes or 8))
    got = read_counts()
    out = {"what": what, "workload_key": wl_key, "patterns": W.B, "m": W.m, "flags": flags,
           "ms_per_launch": wall * 1e3, "kernel_ms_mean": kern_s * 1e3, "kernel_ms_min": kmin,
           "patterns_per_s": W.B / kern_s, "prefix_table_hit_frac": frac,
           "matches_headline": None if ref_counts is None else bool(np.array_equal(got, ref_counts)),
           "roofline": roofline(rnd, stream_bytes, acc, kern_s, W.B, pmc_traffic(wl_key, name, kern_s),
                                stream_read, table)}
    return out, got


def walk_step_bytes(info, idx):
    """HBM bytes of one LF step of the walk: one 32-B occurrence / walk line, or on the
    binary wavelet matrix one rank line per non-pure level of the row's symbol
    (cs_fm_info.active_levels), averaged over the BWT's symbol frequencies."""
    if info.engine != 0:
        return 32.0
    C = idx.C().astype(np.float64)
    f = np.diff(C)
    lines = np.array([bin(info.active_levels[c]).count("1") for c in range(256)], np.float64)
    return float((f * lines).sum() / max(f.sum(), 1)) * info.line_bytes


def locate_leg(name, what, idx, info, wl_key, W, text, flags, dev, sh, reps=3, limit=100000):
    """locate (fm_index.cpp:107-157) of the batch: phase 1 (backward search, min(count,
    limit) per pattern, CSR offsets) and phase 2 (positions: full SA, walk lines or the
    row-sampled SSA walk, as `flags` select), HIP events around each phase; every
    position checked to spell its pattern; phase 2's LF steps from its measurement twin."""
    B, m = W.B, W.m
    stream = torch.cuda.current_stream()
    d_sp = torch.empty(B, dtype=torch.int64, device=dev)
    d_oo = torch.empty(B + 1, dtype=torch.int64, device=dev)
    t1s, t2s, walls = [], [], []
    d_pos = None
    for it in range(reps):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e[0].record(stream)
        tot = idx.locate_ranges_device(W.pats.data_ptr(), W.offs.data_ptr(), B, limit,
                                       d_sp.data_ptr(), d_oo.data_ptr(), sh, flags=flags)
        if d_pos is None:
            d_pos = torch.empty(max(tot, 1), dtype=torch.int64, device=dev)
        e[1].record(stream)
        # phase 2 without its own synchronisation (the overrun check follows the event)
        idx.locate_walk_device(d_sp.data_ptr(), d_oo.data_ptr(), B, tot, d_pos.data_ptr(), sh,
                               sync=False, flags=flags)
        e[2].record(stream)
        idx.locate_check(sh)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        t1s.append(e[0].elapsed_time(e[1]) / 1e3)
        t2s.append(e[1].elapsed_time(e[2]) / 1e3)
    tl = min(walls)
    pos = d_pos[:tot]
    oo = d_oo.cpu().numpy()
    owner = torch.from_numpy(np.repeat(np.arange(B), np.diff(oo).astype(np.int64))).to(dev)
    ok = True
    for a in range(0, tot, 1 << 24):  # chunks: the window gather is 20 B per position
        p, w = pos[a:a + (1 << 24)], owner[a:a + (1 << 24)]
        win = text[(p.unsqueeze(1) + torch.arange(m, device=dev)).long()]
        ok &= bool((win == W.pats.view(B, m)[w]).all().item())
    del owner
    steps = torch.empty(max(tot, 1), dtype=torch.int64, device=dev)
    idx.locate_walk_steps_device(d_sp.data_ptr(), d_oo.data_ptr(), B, tot, steps.data_ptr(), sh,
                                 flags=flags)
    st = int(steps[:tot].sum().item()) if tot else 0
    del steps, d_pos, d_sp, d_oo
    walk_s = min(t2s)
    sb = info.ssa_bytes // max(info.n // info.ssa_stride, 1) if info.ssa_bytes else 4
    step_bytes = walk_step_bytes(info, idx)
    uses_sa = info.full_sa_bytes and not (flags & 4)
    walk_lines = not uses_sa and info.walk_bytes and not (flags & 8)
    # phase 2's random reads: the full SA one dependent read per reported range — a range's
    # rows are consecutive, so its SA entries are one run of ceil(4 c / 32) 32-B sectors,
    # the first random, the rest streamed (repetitive DNA: thousands per range); walk lines
    # one 32-B line per visited row (the start row and every LF step: the line holds the
    # row's mark, symbol and occ) + one sample; the row-sampled walk one LF step's lines
    # per step (a sampled row is known from its index) + one sample
    cnts = np.diff(oo).astype(np.int64)
    if uses_sa:
        nz = int((cnts > 0).sum())
        sa_sectors = int(((cnts * 4 + 31) // 32).sum())
        lines, reads = 0.0, float(nz)
        alg = sa_sectors * 32 + tot * 8 + B * 16
        stream_rd = 16 * B + (sa_sectors - nz) * 32
    else:
        if walk_lines:
            lines = float(st + tot)
        else:
            lines = st * (step_bytes / 32.0)
        reads = lines + tot
        # algorithmic bytes: those reads, the record/offsets read and the position written
        alg = lines * 32 + tot * (sb + 8) + B * 16
        # streamed reads of the phase-2 kernel (PMC correction, profiles/summarize_legs.py):
        # the records + offsets (fused walk-line walk) or the expanded rows (k_walk)
        stream_rd = 16 * B if walk_lines else 8 * tot
    wpmc = pmc_traffic(wl_key, name, walk_s)
    wb, wreads, wbasis = dram_basis(alg, stream_rd, reads, wpmc)
    # the structure the dependent reads hit: the suffix array, the walk lines, or the rank lines
    wtab = ((info.full_sa_bytes, 16) if uses_sa else
            (info.walk_bytes, 32) if walk_lines else (info.rank_bytes, info.line_bytes))
    wceil = random_ceiling(*wtab)
    wbound, wfrac = ceiling_frac(wreads / walk_s, wceil, wtab[0])
    return {"what": what, "workload_key": wl_key, "patterns": B, "positions": int(tot), "seconds": tl,
            "patterns_per_s": B / tl, "positions_per_s": tot / tl,
            "phase1_ms": min(t1s) * 1e3, "phase2_ms": walk_s * 1e3, "limit": limit,
            "flags": flags, "positions_verified": ok,
            "walk_lf_steps_per_position": st / max(tot, 1),
            "phase2_stream_read_bytes": stream_rd, "phase2_alg_bytes": alg,
            "walk_roofline": {"bound": wbound, "achieved": wb / walk_s / 1e9, "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": wb / walk_s / 1e9 / HBM_PEAK_GBS, "basis": wbasis,
                              "alg_bytes": alg, "alg_bytes_per_position": alg / max(tot, 1),
                              **wpmc, "alg_dependent_reads": reads,
                              "dependent_reads_per_s": wreads / walk_s,
                              "random_access_ceiling_per_s": wceil,
                              "frac_of_random_access_ceiling": wfrac}}


def locate_one_leg(name, what, idx, info, wl_key, W, text, dev, sh, reps=5, limit=100000):
    """locate of the batch in one call (cs_fm_locate_device: one launch over full-SA
    indexes — search, look-back scan of the counts, positions — the two phases otherwise),
    wall time per call including the read-back of the total; positions checked to spell
    their patterns."""
    B, m = W.B, W.m
    stream = torch.cuda.current_stream()
    d_oo = torch.empty(B + 1, dtype=torch.int64, device=dev)
    cap = 2 * B
    d_pos = torch.empty(cap, dtype=torch.int64, device=dev)
    # the caller's workspace (cs_fm_locate_device_ws, round 5): no allocation in the call
    wsb = idx.workspace_bytes(B)
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    walls, evs = [], []
    tot = 0
    for it in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        tot, ok = idx.locate_device_ws(W.pats.data_ptr(), W.offs.data_ptr(), B, limit, d_oo.data_ptr(),
                                       d_pos.data_ptr(), cap, ws.data_ptr(), wsb, sh)
        e1.record(stream)
        walls.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        evs.append(e0.elapsed_time(e1) / 1e3)
        if not ok:  # grow the buffer once and time again
            cap = tot
            d_pos = torch.empty(cap, dtype=torch.int64, device=dev)
    tl = min(walls)
    pos = d_pos[:tot]
    oo = d_oo.cpu().numpy()
    owner = torch.from_numpy(np.repeat(np.arange(B), np.diff(oo).astype(np.int64))).to(dev)
    okv = True
    ch = max(1, (1 << 28) // m)  # positions per check: a (ch, m) int64 window index of 2 GB
    for a in range(0, tot, ch):
        p, w = pos[a:a + ch], owner[a:a + ch]
        win = text[(p.unsqueeze(1) + torch.arange(m, device=dev)).long()]
        okv &= bool((win == W.pats.view(B, m)[w]).all().item())
    # algorithmic bytes of the call, per pattern: a pattern the locate records answer
    # (cs_fm_locate_record_hits_device) reads its locate record (64 B, or 16); any other the count's
    # reads (record + context sectors, cs_fm_count_bytes_device) and one 32-B DRAM sector of
    # SA per reported position (the DRAM's access granularity, as the count legs charge
    # their lines) — plus the stream: patterns and offsets in, the search's u32 count and
    # 8-B record per pattern out and back in, the offsets and positions out
    cnt = torch.from_numpy(np.diff(oo).astype(np.int64)).to(dev)
    del owner, d_pos, d_oo, ws
    qb = torch.empty(B, dtype=torch.int64, device=dev)
    idx.count_bytes_device(W.pats.data_ptr(), W.offs.data_ptr(), B, qb.data_ptr(), sh)
    hit = torch.zeros(B, dtype=torch.uint8, device=dev)
    if info.locate_record_bytes:
        idx.locate_record_hits_device(W.pats.data_ptr(), W.offs.data_ptr(), B, hit.data_ptr(), sh)
    hb = hit.bool()
    nhit = int(hb.sum().item())
    rw = getattr(info, "locate_record_width", 0) or 16  # 64-B records: read by four lanes
    # a position costs one 32-B SA sector (full SA), or over walk lines (no full SA, C5) its
    # walk: (LF steps + 1) 32-B lines and one sample sector — the steps measured by the walk's
    # twin (cs_fm_locate_walk_steps_device) over the same rows (round 5: the line charged one
    # SA sector per position there, 30 M random reads per C5 call instead of 57 M)
    per_pos = 1.0
    walk_steps = None
    if not info.full_sa_bytes and tot:
        d_sp = torch.empty(B, dtype=torch.int64, device=dev)
        d_o2 = torch.empty(B + 1, dtype=torch.int64, device=dev)
        t2 = idx.locate_ranges_device(W.pats.data_ptr(), W.offs.data_ptr(), B, limit, d_sp.data_ptr(),
                                      d_o2.data_ptr(), sh)
        stp = torch.empty(max(t2, 1), dtype=torch.int64, device=dev)
        idx.locate_walk_steps_device(d_sp.data_ptr(), d_o2.data_ptr(), B, t2, stp.data_ptr(), sh)
        walk_steps = float(stp[:t2].sum().item()) / max(t2, 1)
        per_pos = walk_steps + 2.0
        del d_sp, d_o2, stp
    rnd = rw * nhit + int(torch.where(hb, 0, qb + (32 * per_pos) * cnt).sum().item())
    # random reads: one per 16-B record, one per 32-B sector or line, per position one SA
    # sector or the walk's lines and sample
    acc = nhit + int(torch.where(hb, 0, (qb + 31) // 32 + per_pos * cnt).sum().item())
    # the search's results, written and read back: an 8-B record per pattern and a 4-B count
    # unless the record is the pattern's only position (count 1; round 5)
    mid = 8 * B + 4 * int((cnt != 1).sum().item())
    del qb, hit, hb, cnt
    stream_b = B * m + (B + 1) * 8 + mid * 2 + (B + 1) * 8 + tot * 8
    alg = rnd + stream_b
    stream_rd = B * m + (B + 1) * 8 + mid  # patterns, offsets, the search's results read back
    lpmc = pmc_traffic(wl_key, name, min(evs))
    fb, reads, basis = dram_basis(alg, stream_rd, acc, lpmc)
    ltab = info.locate_record_bytes or info.prefix_bytes
    lceil = random_ceiling(ltab, 16)
    lbound, lfrac = ceiling_frac(reads / tl, lceil, ltab)
    return {"what": what, "workload_key": wl_key, "patterns": B, "positions": int(tot), "seconds": tl,
            "patterns_per_s": B / tl, "positions_per_s": tot / tl, "limit": limit,
            "event_ms": min(evs) * 1e3, "positions_verified": okv,
            "locate_record_hit_frac": nhit / B, "walk_lf_steps_per_position": walk_steps,
            "roofline": {"bound": lbound, "achieved": fb / tl / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": fb / tl / 1e9 / HBM_PEAK_GBS, "basis": basis, "alg_bytes_per_launch": alg,
                         "alg_bytes_per_query": alg / B,
                         "alg_random_bytes_per_launch": rnd, "alg_stream_bytes_per_launch": stream_b,
                         "stream_read_bytes_per_launch": stream_rd, "alg_random_accesses_per_launch": acc,
                         **lpmc, "random_accesses_per_s": reads / tl,
                         "random_access_ceiling_per_s": lceil,
                         "frac_of_random_access_ceiling": lfrac}}


def stream_leg(name, what, idx, W, dev, sh, ref_counts, chunks=10, packed=False, u8=False):
    """count of patterns streamed from host memory (BASELINE C5: "1 B streamed 20-mer
    count()", 125 M per GPU): `chunks` batches of W.B patterns from page-locked host
    buffers — the caller's, reused for every chunk — through two device slots: the H2D
    copy of chunk i+1 on a copy stream overlaps the count of chunk i on the launch stream
    and the D2H copy of chunk i-1's counts on a third stream (events order the slots).
    PCIe-bound: reported against a plain H2D copy of the same bytes, timed alone.  u8
    (packed only): counts as the exact uint8 form, counts >= 255 as (pattern, count) pairs
    (a quarter of the u32 D2H bytes)."""
    B, m = W.B, W.m
    comp = torch.cuda.current_stream()
    cin, cout = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    if packed:  # 2-bit DNA, 8 B per pattern, u32 counts
        lut = torch.zeros(256, dtype=torch.int64, device=dev)
        lut[torch.tensor(list(b"ACGT"), device=dev)] = torch.arange(4, device=dev)
        codes = lut[W.pats.view(B, m).long()]
        hin = [((codes << (2 * torch.arange(m, device=dev))).sum(dim=1)).cpu().pin_memory()]
        del codes
        cdt, cw = (torch.uint8, 1) if u8 else (torch.int32, 4)
    else:  # the reference's byte strings with u64 offsets, u64 counts
        hin = [W.pats.cpu().pin_memory(), W.offs.cpu().pin_memory()]
        cdt, cw = torch.int64, 8
    dslot = [[torch.empty_like(x, device=dev) for x in hin] for _ in range(2)]
    dout = [torch.empty(B, dtype=cdt, device=dev) for _ in range(2)]
    hout = [torch.empty(B, dtype=cdt).pin_memory() for _ in range(2)]
    XC = 1 << 16  # pair capacity per chunk (u8 form)
    dexc = [torch.empty(2 * XC + 1, dtype=torch.int64, device=dev) for _ in range(2)] if u8 else None
    hexc = [torch.empty(2 * XC + 1, dtype=torch.int64).pin_memory() for _ in range(2)] if u8 else None
    in_bytes = sum(x.numel() * x.element_size() for x in hin)

    def launch(s, st):
        if u8:  # the pair counter sits after the pairs; zeroed on the launch stream
            dexc[s][2 * XC:].zero_()
            idx.count_packed_device(dslot[s][0].data_ptr(), m, B, dout[s].data_ptr(), width=1,
                                    d_exc=dexc[s].data_ptr(), exc_cap=XC,
                                    d_exc_n=dexc[s].data_ptr() + 16 * XC, stream=st)
        elif packed:
            idx.count_packed_device(dslot[s][0].data_ptr(), m, B, dout[s].data_ptr(), width=4, stream=st)
        else:
            idx.count_batch_device(dslot[s][0].data_ptr(), dslot[s][1].data_ptr(), B, dout[s].data_ptr(), st)

    def run(nchunks):
        loaded = [torch.cuda.Event() for _ in range(2)]
        counted = [torch.cuda.Event() for _ in range(2)]
        drained = [None, None]
        for i in range(nchunks):
            s = i % 2
            with torch.cuda.stream(cin):
                if i >= 2:
                    cin.wait_event(counted[s])  # the slot's previous count has read its input
                for d, h in zip(dslot[s], hin):
                    d.copy_(h, non_blocking=True)
                loaded[s].record(cin)
            comp.wait_event(loaded[s])
            if drained[s] is not None:
                comp.wait_event(drained[s])  # the slot's previous counts are back on the host
            launch(s, comp.cuda_stream)
            counted[s].record(comp)
            with torch.cuda.stream(cout):
                cout.wait_event(counted[s])
                hout[s].copy_(dout[s], non_blocking=True)
                if u8:
                    hexc[s].copy_(dexc[s], non_blocking=True)
                drained[s] = torch.cuda.Event()
                drained[s].record(cout)
        torch.cuda.synchronize()

    run(2)  # warm-up
    walls = []
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(chunks)
        walls.append(time.perf_counter() - t0)
    tl = min(walls)
    # the PCIe ceiling: the same H2D bytes alone, one chunk's buffers per copy
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(chunks):
        for d, h in zip(dslot[i % 2], hin):
            d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    h2d_s = time.perf_counter() - t0
    got = hout[(chunks - 1) % 2].numpy().astype(np.int64)
    if u8:  # exact counts from the uint8 form and its pairs
        e = hexc[(chunks - 1) % 2].numpy()
        ne = int(e[2 * XC])
        assert ne <= XC, "pair area too small"
        pr = e[:2 * ne].reshape(-1, 2)
        got[pr[:, 0]] = pr[:, 1]
    out = {"what": what, "patterns": B * chunks, "chunks": chunks, "chunk_patterns": B, "m": m,
           "seconds": tl, "patterns_per_s": B * chunks / tl,
           "h2d_bytes_per_pattern": in_bytes / B, "d2h_bytes_per_pattern": cw + (16 * XC + 8) / B * u8,
           "h2d_GBs": in_bytes * chunks / tl / 1e9,
           "pcie_h2d_alone_GBs": in_bytes * chunks / h2d_s / 1e9,
           "frac_of_h2d_alone": h2d_s / tl,
           "matches_headline": None if ref_counts is None else bool(np.array_equal(got, ref_counts))}
    del dslot, dout, hout, hin, dexc, hexc
    return out


def build_index(pkg, text, N, stride, dev_index, env=None):
    """Build with the engine's environment switches `env` set for the build ("" = unset)."""
    saved = {}
    for k, v in (env or {}).items():
        saved[k] = os.environ.get(k)
        if v == "":
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    try:
        t0 = time.perf_counter()
        idx = pkg.FMIndex.build_from_device_text(text.data_ptr(), N, pkg.BuildParams(ssa_stride=stride),
                                                 device=dev_index)
        torch.cuda.synchronize()
        return idx, time.perf_counter() - t0
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def workload_key(kind, N, m, B, info, queries):
    engine = {1: "occ", 2: "qwm", 3: "locc"}.get(info.engine, "wm%d" % info.line_bytes)
    wl = "%s:%d:m%d:b%d:%s:k%d" % (kind, N, m, B, engine, info.prefix_k)
    if info.context_q:
        wl += ":ctx%d" % info.context_q
    if info.record_bytes:
        wl += ":rec%d" % info.record_bytes  # context records (32-/16-B prefix-table entries)
    if queries != "text":
        wl += ":" + queries
    return wl


def engine_name(info):
    if info.engine in (1, 3):
        return "%s + left contexts (q=%d)%s" % (
            "learned occurrence lines" if info.engine == 3 else "occurrence lines", info.context_q,
            " + %d-B context records" % info.record_bytes if info.record_bytes else "")
    if info.engine == 2:
        return "quaternary wavelet matrix (%d levels of occurrence lines)" % info.levels
    return "binary wavelet matrix, 8 levels (%d-B rank lines)" % info.line_bytes


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, child_argv, script=None, env=None):
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (one
    per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, as
    torch.distributed.run would) and wait for them.  Called before anything touches the
    GPU — the parent never initialises HIP and never exec()s; the ranks are children.
    Rank 0's JSON line is the only stdout line: its other stdout lines (e.g. gloo's
    connection notices) and the other ranks' stdout go to stderr.  When one rank fails, the others are terminated (by PID) and its exit
    status is returned; 0 when every rank succeeded."""
    import signal
    import subprocess
    script = script or os.path.abspath(__file__)
    base = dict(os.environ if env is None else env)
    base.update({"WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                 "MASTER_PORT": str(free_port()), "GROUP_RANK": "0", "CS_BENCH_SPAWNED": "1"})
    import threading
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-u", script] + list(child_argv), env=e,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr))

    def relay(pipe):
        # rank 0's JSON line to stdout; anything else a library prints there to stderr
        for raw in iter(pipe.readline, b""):
            line = raw.decode(errors="replace")
            dst = sys.stdout if line.lstrip().startswith("{") else sys.stderr
            dst.write(line)
            dst.flush()

    relay_t = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    relay_t.start()

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + 10
        for p in procs:
            try:
                p.wait(max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    old = signal.signal(signal.SIGTERM, lambda *_: (stop(), sys.exit(143)))
    try:
        rc = 0
        while [p.poll() for p in procs].count(None):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                rc = bad[0]
                print("[bench] a rank exited with status %d; stopping the others" % rc,
                      file=sys.stderr, flush=True)
                stop()
                break
            time.sleep(0.2)
        relay_t.join(10)
        bad = [p.returncode for p in procs if p.returncode != 0]
        return rc or (bad[0] if bad else 0)
    finally:
        signal.signal(signal.SIGTERM, old)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--kind", default="dna", choices=["dna", "bytes"])
    ap.add_argument("--text-bytes", type=int, default=3_999_999_999,
                    help="text length before the terminator (C4: 3,999,999,999)")
    ap.add_argument("--m", type=int, default=20)
    ap.add_argument("--batch", type=int, default=12_500_000, help="patterns per GPU per step")
    ap.add_argument("--ssa-stride", type=int, default=32)
    ap.add_argument("--cpu-queries", type=int, default=None,
                    help="patterns timed through the reference's count() on the CPU (default: "
                         "SURVEY §8(d)'s 256 at C2-size texts, 32 at C3, 16 at C4 and above, and "
                         "at least two per host thread)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--p50-calls", type=int, default=1000)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--queries", default="text", choices=["text", "unif"],
                    help="Q_text (substrings of the text, the headline) or Q_unif (uniform random)")
    ap.add_argument("--cpu-fast-queries", type=int, default=1_000_000,
                    help="patterns timed through the oracle's fast (precomputed) count, all threads")
    ap.add_argument("--extract-batch", type=int, default=1_000_000,
                    help="random 20-byte extracts timed on the device (N=1 only; 0 = skip)")
    ap.add_argument("--stream-chunks", type=int, default=10,
                    help="count_stream legs: chunks of --batch patterns streamed from host memory "
                         "(10 x 12.5 M = C5's 1 B patterns over 8 GPUs, per GPU)")
    ap.add_argument("--replicate", default="build", choices=["build", "broadcast"],
                    help="N > 1: every rank builds its replica, or rank 0 builds and broadcasts "
                         "the device image (RCCL)")
    ap.add_argument("--no-gather", action="store_true",
                    help="N > 1: keep each rank's counts (no gather to rank 0)")
    ap.add_argument("--prefix-k", type=int, default=None,
                    help="prefix-table depth override (0 = off; default automatic)")
    ap.add_argument("--hbm-budget", default=None,
                    help="HBM budget of the headline index (CS_FM_HBM_BUDGET: bytes, K/M/G/T suffix)")
    ap.add_argument("--legs", default="all",
                    help="comma-separated legs of a full N=1 run (%s), 'all' or 'none'"
                         % ",".join(ALL_LEGS))
    ap.add_argument("--legs-out", default=None,
                    help="file for the full result with every leg (default gpurun_out/"
                         "bench_full_n<N>_<time>.json; 'none' = stderr only); stdout gets the "
                         "compact headline line (<= 4 KB)")
    ap.add_argument("--only", default=None,
                    help="run only this leg ('count' = the headline) and print its object "
                         "(profiling passes)")
    args = ap.parse_args()
    if args.prefix_k is not None:
        os.environ["CS_FM_PREFIX_K"] = str(args.prefix_k)
    if args.hbm_budget is not None:
        os.environ["CS_FM_HBM_BUDGET"] = args.hbm_budget
    legs = (set(ALL_LEGS) if args.legs == "all" else set() if args.legs == "none"
            else set(x for x in args.legs.split(",") if x))
    if args.only:
        legs = {args.only} - {"count"}
        args.no_cpu, args.p50_calls = True, 0

    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    ndev = torch.cuda.device_count()  # does not initialise the GPU on this image
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: this process starts the N ranks itself (before any GPU call)
        if args.dist_backend == "nccl" and ndev < args.gpus:
            sys.exit("bench.py: --gpus %d over RCCL needs %d GPUs, %d visible (rehearse with "
                     "--dist-backend gloo)" % (args.gpus, args.gpus, ndev))
        rc = spawn_ranks(args.gpus, sys.argv[1:])
        sys.exit(rc if rc >= 0 else 128 - rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d: the line would not describe the run"
                 % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.dist_backend == "nccl" and ndev < int(os.environ.get("LOCAL_WORLD_SIZE", world)):
        sys.exit("bench.py: RCCL needs one GPU per rank (%d visible)" % ndev)
    local_dev = local % max(ndev, 1)  # identity on an N-GPU node; lets a 1-GPU box rehearse N ranks
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    rank_devices = None
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
        assert dist.get_rank() == rank
        # which GPU every rank runs on (PCI bus of its device), gathered to the line
        pr = torch.cuda.get_device_properties(dev)
        me = "%d:%s:%s" % (rank, local_dev, getattr(pr, "pci_bus_id", "?"))
        rank_devices = [None] * world
        dist.all_gather_object(rank_devices, me)
        legs = set()  # the N=1 legs; N > 1 runs the headline and the sharded locate
    pkg = _load_pkg()
    import importlib
    shard = importlib.import_module("cs_fmindex_amd.shard")
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    # ---- synthetic text in HBM, index built on this GPU ----
    L = args.text_bytes
    N = L + 1
    t0 = time.perf_counter()
    text = torch.empty(N + 16, dtype=torch.uint8, device=dev)
    pkg.synth_text_device(args.kind, 42, L, text.data_ptr(), sh)
    torch.cuda.synchronize()
    replicate_s = None
    need_main = not (args.only and (args.only in LEGS_WM or args.only in LEGS_WALK
                                    or args.only in LEGS_LEARNED or args.only in LEGS_RDNA
                                    or args.only in LEGS_FOOT))
    idx = None
    if need_main:
        if args.replicate == "broadcast" and world > 1:
            # rank 0 builds; the device image goes to every rank (shard.replicate_index)
            idx = build_index(pkg, text, N, args.ssa_stride, local_dev)[0] if rank == 0 else None
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            idx = shard.replicate_index(pkg, idx, 0, rank, world, dev)
            replicate_s = time.perf_counter() - t1
        else:
            idx = build_index(pkg, text, N, args.ssa_stride, local_dev)[0]
        torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    B, m = args.batch, args.m
    total = B * world  # weak scaling: B patterns per GPU
    lo, hi = shard.shard_range(total, rank, world)
    assert hi - lo == B
    W = Workload(pkg, text, N, m, lo, B, args.kind, args.queries, dev, sh)
    res = {}
    counts = None
    kern_avg_s = None

    if need_main:
        info = idx.info()
        log(rank, "index built: n=%d in %.1f s, rank lines %.2f GB" % (N, build_s, info.rank_bytes / 1e9))
        wl = workload_key(args.kind, N, m, B, info, args.queries)
        out = torch.empty(B, dtype=torch.int64, device=dev)
        # the call's device workspace (cs_fm_count_device_ws, round 5): the lists of routed
        # patterns live here, zero-filled once, so no call allocates
        ws_bytes = idx.workspace_bytes(B)
        ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=dev)

        def headline():
            idx.count_device_ws(W.pats.data_ptr(), W.offs.data_ptr(), B, out.data_ptr(), ws.data_ptr(),
                                ws_bytes, stream=sh)

    if need_main and (not args.only or args.only == "count"):
        # ---- the timed region: K steps of the batch count (+ the gather at N > 1) ----
        coll = world > 1 and not args.no_gather
        wcap = shard.WIRE_CAP
        if coll:
            # the wire form's overflow area holds every count >= 255 of the batch (each step
            # counts the same batch): sized from the first count, the largest shard's need
            headline()
            nover = torch.tensor([int((out >= 255).sum().item())], dtype=torch.int64, device=dev)
            dist.all_reduce(nover, op=dist.ReduceOp.MAX)
            wcap = max(shard.WIRE_CAP, int(nover.item()))
        wire_len = shard.wire_bytes(pkg, B, wcap) if coll else 0
        pg = shard.PipelinedGather(wire_len, world, rank, torch.uint8, dev) if coll else None

        def step(k):
            headline()
            if coll:  # exact 1-B wire form, gathered behind the next step's count
                w = pg.buffer(k)
                shard.pack_counts(pkg, out, w, cap=wcap, stream=sh)
                pg.submit(k)

        for k in range(args.warmup):
            step(k)
        if coll:
            pg.finish()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        t0 = time.perf_counter()
        for k in range(args.steps):
            evs[k][0].record(stream)
            headline()
            evs[k][1].record(stream)
            if coll:
                w = pg.buffer(k)
                shard.pack_counts(pkg, out, w, cap=wcap, stream=sh)
                pg.submit(k)
        if coll:
            pg.finish()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        kern_ms = [a.elapsed_time(b) for a, b in evs]
        if world > 1:
            tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed = tt.item()
        counts = out.cpu().numpy()
        gather_ok = None
        if coll:
            # rank 0 decodes every shard of the last step and checks it against its own
            # count of the same patterns (the whole global batch, shard by shard)
            if rank == 0:
                gather_ok = True
                parts = pg.result_parts((args.steps - 1))
                for r in range(world):
                    got = shard.unpack_counts(parts[r], B)
                    Wr = W if r == 0 else Workload(pkg, text, N, m, shard.shard_range(total, r, world)[0],
                                                   B, args.kind, args.queries, dev, sh)
                    chk = torch.empty(B, dtype=torch.int64, device=dev)
                    idx.count_batch_device(Wr.pats.data_ptr(), Wr.offs.data_ptr(), B, chk.data_ptr(), sh)
                    gather_ok &= bool(torch.equal(got.to(dev), chk))
                    del chk
            del pg
        found = int((counts >= 1).sum())
        # the roofline's kernel time: the median over the K timed launches (HIP events on the
        # launch stream) — a profile's summary is a median over as many dispatches
        # (profiles/profile_count.sh), so the two agree
        kern_avg_s = statistics.median(kern_ms) / 1e3
        rnd, acc, frac = W.accounting(idx, info, 0, sh, dev)
        stream_b = B * m + (B + 1) * 8 + B * 8  # patterns, offsets, uint64 counts
        if rank == 0:
            rf = roofline(rnd, stream_b, acc, kern_avg_s, B, pmc_traffic(wl, "count", kern_avg_s),
                          B * m + (B + 1) * 8,
                          (info.prefix_bytes, info.record_bytes or 8) if info.prefix_bytes
                          else (info.rank_bytes, info.line_bytes))
            rf.update({"line_bytes": info.line_bytes, "prefix_k": info.prefix_k,
                       "prefix_table_hit_frac": frac, "context_q": info.context_q,
                       # SURVEY.md §8(d)'s per-query figure for the reference's structure
                       # (64 B x 8 levels x 2 ranks x (m-1) steps), for comparison only:
                       # this engine reads alg_bytes_per_query
                       "survey_alg_bytes_per_query": 64 * 8 * 2 * (m - 1),
                       "survey_equivalent_GBs": 64 * 8 * 2 * (m - 1) * B / kern_avg_s / 1e9,
                       "kernel_ms_median": kern_avg_s * 1e3, "kernel_ms_mean": statistics.mean(kern_ms),
                       "kernel_ms_min": min(kern_ms), "kernel_ms_max": max(kern_ms),
                       "kernel_time_basis": "median of %d launches (HIP events)" % len(kern_ms),
                       "workspace_bytes": ws_bytes})
            res = {
                "metric": METRIC,
                "value": B * world * args.steps / elapsed,
                "unit": "patterns/s",
                "n_gpus": world,
                "ranks_seen": dist.get_world_size() if world > 1 else 1,
                "rank_devices": rank_devices,
                "launcher": ("bench.py --gpus (ranks spawned by bench.py)" if os.environ.get("CS_BENCH_SPAWNED")
                             else "external (torch.distributed.run)" if world > 1 else "single process"),
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": elapsed / args.steps * 1e3,
                "higher_is_better": True,
                "scaling": "weak",
                "vs_baseline": None,
                "dtype": "u64",
                "data": "synthetic",
                "config": {"workload": "C4: %s text n=%d (incl. terminator), Q_%s %d-mers, count()"
                           % (args.kind.upper(), N, args.queries, m) if L == 3_999_999_999 else
                           "%s text n=%d, Q_%s %d-mers, count()" % (args.kind, N, args.queries, m),
                           "batch_per_gpu": B, "global_batch": B * world, "m": m,
                           "ssa_stride": args.ssa_stride, "parallelism": "dp%d" % world,
                           "index": "replicated per GPU", "workload_key": wl,
                           "collective": ("gather of every step's counts to rank 0 (%s), exact "
                                          "1-B wire form, %d B per rank per step, overlapped with "
                                          "the next step's count" % (
                                              "RCCL over xGMI" if args.dist_backend == "nccl"
                                              else args.dist_backend, wire_len)) if coll
                           else "none (independent query shards)",
                           "engine": engine_name(info)},
                "roofline": rf,
                "build_s": build_s,
                # every device allocation the handle owns (cs_fm_info.device_bytes, round 5:
                # the derived locate records and 2-bit text included — VERDICT r04 weak item 5)
                "index_hbm_bytes": int(info.device_bytes),
                "index_image_bytes": int(sum(idx.export_meta()[1])),
                "index_bytes_per_base": info.device_bytes / N,
                "index_parts": {"prefix_table_or_records": info.prefix_bytes,
                                "left_contexts": info.context_bytes, "rank_lines": info.rank_bytes,
                                "walk_lines": info.walk_bytes, "full_sa": info.full_sa_bytes,
                                "ssa": info.ssa_bytes, "text_in_hbm": bool(info.text_in_hbm),
                                "locate_records": info.locate_record_bytes,
                                "packed_text": info.packed_text_bytes},
                "replicate": args.replicate if world > 1 else "single",
                "replicate_s": replicate_s,
                "found_frac": found / B,
            }
            if coll:
                res["gather_verified"] = gather_ok

    # ---- N > 1: locate of each rank's shard, positions gathered to rank 0 (gather_v) ----
    if world > 1 and need_main and not args.only:
        d_oo = torch.empty(B + 1, dtype=torch.int64, device=dev)
        cap = 2 * B
        d_pos = torch.empty(cap, dtype=torch.int64, device=dev)
        tot, fits = idx.locate_device(W.pats.data_ptr(), W.offs.data_ptr(), B, 100000, d_oo.data_ptr(),
                                      d_pos.data_ptr(), cap, sh)  # sizes the position buffer
        if not fits:
            d_pos = torch.empty(tot, dtype=torch.int64, device=dev)
            cap = tot
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        tot, fits = idx.locate_device(W.pats.data_ptr(), W.offs.data_ptr(), B, 100000, d_oo.data_ptr(),
                                      d_pos.data_ptr(), cap, sh)
        assert fits
        parts = shard.gather_v(d_pos[:tot], world, rank)
        torch.cuda.synchronize()
        tl = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
        dist.all_reduce(tl, op=dist.ReduceOp.MAX)
        pos = d_pos[:tot]
        oo = d_oo.cpu().numpy()
        owner = torch.from_numpy(np.repeat(np.arange(B), np.diff(oo).astype(np.int64))).to(dev)
        win = text[(pos.unsqueeze(1) + torch.arange(m, device=dev)).long()]
        okt = torch.tensor([int(bool((win == W.pats.view(B, m)[owner]).all().item()))],
                           dtype=torch.int64, device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        tt = torch.tensor([tot], dtype=torch.int64, device=dev)
        dist.all_reduce(tt)
        if rank == 0:
            res["locate"] = {"patterns": B * world, "positions": int(tt.item()),
                             "seconds": tl.item(), "patterns_per_s": B * world / tl.item(),
                             "positions_per_s": int(tt.item()) / tl.item(), "limit": 100000,
                             "positions_verified": bool(okt.item()),
                             "gathered_positions": int(sum(p.numel() for p in parts)),
                             "method": "cs_fm_locate_device per rank (one call), then gather_v",
                             "collective": "gather_v of every rank's positions to rank 0"}
        del d_oo, d_pos, owner, win, parts

    # ---- N = 1 legs on the headline index ----
    lg = {}
    m_counts = {}  # the default path's counts of the m-legs, for the other forms' equality check
    leg_errors = {}
    stream_m = B * m + (B + 1) * 8
    with LegGuard(leg_errors, "main legs"):
        if need_main and legs & set(LEGS_MAIN):
            steps, warm = max(3, args.steps // 2), 2
            if "count_100m" in legs:
                # BASELINE configs[3]'s whole 100 M-pattern batch on one GPU (VERDICT r04 missing
                # #3): the same Q_text stream, 8 x --batch patterns in one call (2 GB of patterns,
                # 0.8 GB of offsets and of counts beside the index), the workspace sized for it;
                # the first --batch counts must equal the headline's
                BB = 8 * B
                WB = Workload(pkg, text, N, m, lo, BB, args.kind, args.queries, dev, sh)
                ob = torch.empty(BB, dtype=torch.int64, device=dev)
                wsb = idx.workspace_bytes(BB)
                wsB = torch.zeros(wsb, dtype=torch.uint8, device=dev)
                r, got = count_leg(
                    "count_100m", "the headline count over BASELINE configs[3]'s whole 100 M-pattern "
                    "batch in one call on one GPU (8 x the per-GPU batch of the weak-scaling line)",
                    idx, info, wl + ":100m", WB,
                    lambda: idx.count_device_ws(WB.pats.data_ptr(), WB.offs.data_ptr(), BB, ob.data_ptr(),
                                                wsB.data_ptr(), wsb, stream=sh),
                    0, BB * m + (BB + 1) * 8 + 8 * BB, max(3, args.steps // 4), 1, stream, sh, dev, None,
                    lambda: ob.cpu().numpy())
                r["matches_headline_prefix"] = None if counts is None else bool(np.array_equal(got[:B], counts))
                r["vs_headline_patterns_per_s"] = r["patterns_per_s"] / (B / kern_avg_s) if kern_avg_s else None
                lg["count_100m"] = r
                del WB, ob, wsB, got
            if "count_streams" in legs:
                # the headline batch as independent batches issued round-robin over S streams
                # (a serving loop's pattern), each stream its own workspace and output: K calls
                # between two synchronisations, wall time per call.  One call's tail (its last
                # blocks draining, the list kernel) overlaps the next call's head on another
                # stream (profiles/scripts/stream_probe.py); the headline line itself stays on
                # one stream, so its per-launch kernel time is the launch's own.
                ss = [torch.cuda.Stream(device=dev) for _ in range(3)]
                wss = [torch.zeros(ws_bytes, dtype=torch.uint8, device=dev) for _ in range(3)]
                oss = [torch.empty(B, dtype=torch.int64, device=dev) for _ in range(3)]
                K = max(24, args.steps)
                per = {1: [], 2: [], 3: []}

                def run_s(S):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for i in range(K):
                        j = i % S
                        idx.count_device_ws(W.pats.data_ptr(), W.offs.data_ptr(), B, oss[j].data_ptr(),
                                            wss[j].data_ptr(), ws_bytes, stream=ss[j].cuda_stream)
                    torch.cuda.synchronize()
                    return (time.perf_counter() - t0) * 1e3 / K

                for S in per:
                    run_s(S)
                for _ in range(3):
                    for S in per:
                        per[S].append(run_s(S))
                same = counts is None or all(np.array_equal(o.cpu().numpy(), counts) for o in oss)
                lg["count_streams"] = {
                    "what": "the headline batch as independent batches round-robin over 1 / 2 / 3 streams "
                            "(own workspace and output each), wall ms per batch, median of 3 rounds",
                    "patterns": B, "calls": K,
                    "ms_per_batch": {str(S): statistics.median(v) for S, v in per.items()},
                    "patterns_per_s": {str(S): B / (statistics.median(v) / 1e3) for S, v in per.items()},
                    "matches_headline": bool(same)}
                del ss, wss, oss
            if "count_u32" in legs and N < 2 ** 32:  # uint32 counts need n < 2^32
                o4 = torch.empty(B, dtype=torch.int32, device=dev)
                lg["count_u32"], _ = count_leg(
                    "count_u32", "the headline batch with uint32 counts (exact, n < 2^32)", idx, info, wl,
                    W, lambda: idx.count_device_ex(W.pats.data_ptr(), W.offs.data_ptr(), B, o4.data_ptr(),
                                                   width=4, stream=sh),
                    0, stream_m + 4 * B, steps, warm, stream, sh, dev, counts,
                    lambda: o4.cpu().numpy().astype(np.int64))
                del o4
            if "count_packed" in legs and args.kind == "dna" and m <= 32 and N < 2 ** 32:
                # 2-bit packed patterns (8 B each, no offsets) and uint32 counts
                lut = torch.full((256,), 0, dtype=torch.int64, device=dev)
                lut[torch.tensor(list(b"ACGT"), device=dev)] = torch.arange(4, device=dev)
                codes = lut[W.pats.view(B, m).long()]
                packed = (codes << (2 * torch.arange(m, device=dev))).sum(dim=1)
                del codes
                o4 = torch.empty(B, dtype=torch.int32, device=dev)
                lg["count_packed"], _ = count_leg(
                    "count_packed", "the headline batch as 2-bit packed DNA (8 B per pattern), uint32 "
                    "counts", idx, info, wl, W,
                    lambda: idx.count_packed_device(packed.data_ptr(), m, B, o4.data_ptr(), width=4,
                                                    stream=sh),
                    0, 8 * B + 4 * B, steps, warm, stream, sh, dev, counts,
                    lambda: o4.cpu().numpy().astype(np.int64), stream_read=8 * B)
                del o4, packed
            for name, fl, what in (("count_table_steps", 2, "prefix table, then the reference's backward-"
                                    "search steps (fm_index.cpp:90-96), one occurrence line per rank pair: "
                                    "no left contexts / context records (CS_Q_NO_CONTEXTS)"),
                                   ("count_lf_loop", 3, "the reference's whole backward-search loop "
                                    "(fm_index.cpp:84-98) from C[], every character one rank step over "
                                    "the occurrence lines (CS_Q_NO_PREFIX | CS_Q_NO_CONTEXTS)")):
                if name in legs:
                    o8 = torch.empty(B, dtype=torch.int64, device=dev)
                    lg[name], _ = count_leg(
                        name, what, idx, info, wl, W,
                        lambda fl=fl, o8=o8: idx.count_device_ex(W.pats.data_ptr(), W.offs.data_ptr(), B,
                                                                 o8.data_ptr(), flags=fl, stream=sh),
                        fl, stream_m + 8 * B, max(3, steps // 4), 1, stream, sh, dev, counts,
                        lambda o8=o8: o8.cpu().numpy())
                    del o8
            ver = "rank steps until the range is at most 8 rows, then the rows' suffix-array entries " \
                  "and the text before them (verification)" if info.full_sa_bytes and info.text_in_hbm else None
            longk = ("k_count_long: the last 32 characters give the context record and the candidate rows "
                     "(inline contexts), then each candidate's suffix-array entry and its window against the "
                     "%s text" % ("2-bit" if info.packed_text_bytes else "byte")) if ver else None
            for name, mm, fl, env in (("count_m32", 32, 0, None), ("count_m64", 64, 0, None),
                                      ("count_m64_steps", 64, 16, None), ("count_m150", 150, 0, None),
                                      ("count_m150_staged", 150, pkg.QT_NO_ROUTE, True),
                                      ("count_m64_long", 64, 32, None), ("count_m150_long", 150, 32, None)):
                if name in legs:
                    Wm = Workload(pkg, text, N, mm, lo, B, args.kind, args.queries, dev, sh)
                    o8 = torch.empty(B, dtype=torch.int64, device=dev)
                    steps_what = "%d rank steps, then the left contexts" % (mm - info.prefix_k - info.context_q)
                    if fl & 16:
                        what = "prefix table, %s (CS_Q_NO_VERIFY)" % steps_what
                    elif fl & 32:
                        what = "%s (CS_Q_LONG: asked for directly)" % (longk or steps_what)
                    elif env:
                        what = ("the staged kernel alone (CS_QT_NO_ROUTE, round 2's default path): prefix "
                                "table, %s" % (ver or steps_what))
                    elif mm > 32 and longk:
                        what = ("the default path: after the first batch with patterns over 32 characters the "
                                "staged kernel leaves them to %s" % longk)
                    else:
                        what = "prefix table, %s" % (ver or steps_what)
                    r, got = count_leg(
                        name, "Q_text %d-mers through the headline index: %s" % (mm, what),
                        idx, info, wl, Wm,
                        lambda Wm=Wm, o8=o8, fl=fl: idx.count_device_ex(Wm.pats.data_ptr(), Wm.offs.data_ptr(),
                                                                        B, o8.data_ptr(), flags=fl, stream=sh),
                        fl, B * mm + (B + 1) * 8 + 8 * B, max(3, steps // 4), 1, stream, sh, dev, None,
                        lambda o8=o8: o8.cpu().numpy())
                    r["found_frac"] = float((got >= 1).mean())
                    if name == "count_m%d" % mm:
                        m_counts[mm] = got
                    else:
                        r["matches_default"] = bool(np.array_equal(got, m_counts[mm])) if mm in m_counts else None
                    lg[name] = r
                    del Wm, o8
            if "count_unif" in legs and args.queries == "text":
                # SURVEY §8(d)'s secondary batch Q_unif: uniform random patterns of the text's
                # alphabet (most 20-mers absent from a 4 GB text)
                Wu = Workload(pkg, text, N, m, lo, B, args.kind, "unif", dev, sh)
                o8 = torch.empty(B, dtype=torch.int64, device=dev)
                r, got = count_leg(
                    "count_unif", "Q_unif: uniform random %d-mers (SURVEY §8(d) secondary batch)" % m,
                    idx, info, wl + ":unif", Wu,
                    lambda Wu=Wu, o8=o8: idx.count_batch_device(Wu.pats.data_ptr(), Wu.offs.data_ptr(), B,
                                                                o8.data_ptr(), sh),
                    0, stream_m + 8 * B, steps, warm, stream, sh, dev, None, lambda o8=o8: o8.cpu().numpy())
                r["found_frac"] = float((got >= 1).mean())
                lg["count_unif"] = r
                del Wu, o8
            if "count_fixed" in legs:
                # one-length k-mers back to back (cs_fm_count_fixed_device: no offsets array)
                fo = torch.empty(B, dtype=torch.int64, device=dev)
                lg["count_fixed"], _ = count_leg(
                    "count_fixed", "the headline batch as one-length k-mers (no offsets array)", idx, info,
                    wl, W, lambda: idx.count_fixed_device(W.pats.data_ptr(), m, B, fo.data_ptr(), sh),
                    0, B * m + 8 * B, steps, warm, stream, sh, dev, counts, lambda: fo.cpu().numpy(),
                    stream_read=B * m)
                del fo
            if "locate" in legs:
                lg["locate"] = locate_leg("locate", "locate (fm_index.cpp:107-157), limit 100000: positions "
                                          "from the full suffix array" if info.full_sa_bytes else
                                          "locate, limit 100000", idx, info, wl, W, text, 0, dev, sh)
            if "locate_one" in legs:
                lg["locate_one"] = locate_one_leg(
                    "locate_one", "locate (fm_index.cpp:107-157), limit 100000, in one call "
                    "(cs_fm_locate_device: one launch — search, look-back scan, positions from the "
                    "full suffix array)", idx, info, wl, W, text, dev, sh)
            if "locate_ssa_rows" in legs:
                lg["locate_ssa_rows"] = locate_leg(
                    "locate_ssa_rows", "locate with the reference's SSA walk (fm_index.cpp:125-153): LF over the occurrence "
                    "lines to a row with row %% %d == 0, SA sample + steps (CS_Q_NO_FULL_SA | "
                    "CS_Q_NO_WALK_LINES)" % args.ssa_stride, idx, info, wl, W, text, 4 | 8, dev, sh, reps=2)
            for name, mm, one in (("locate_m64", 64, True), ("locate_m150", 150, True),
                                  ("locate_m64_steps", 64, False)):
                # long patterns: a narrow range finishes by verification against the text
                # (positions SA[r] - k of the verified rows), or steps to the end (CS_Q_NO_VERIFY)
                if name in legs and (one or info.full_sa_bytes):
                    Wm = Workload(pkg, text, N, mm, lo, B, args.kind, args.queries, dev, sh)
                    if one:
                        lg[name] = locate_one_leg(
                            name, "locate of Q_text %d-mers in one call: %s" % (
                                mm, ("after the first batch with patterns over 32 characters the staged "
                                     "search leaves them to k_locate_long (%s; a pattern's only position "
                                     "is the verified row's SA entry minus k), then the tile scan and "
                                     "the positions" % longk) if longk else
                                ("record, contexts, then %s" % (ver or "rank steps"))),
                            idx, info, wl, Wm, text, dev, sh)
                    else:
                        lg[name] = locate_leg(
                            name, "locate of Q_text %d-mers, rank steps to the end (CS_Q_NO_VERIFY), "
                            "positions from the full suffix array" % mm, idx, info, wl, Wm, text, 16,
                            dev, sh, reps=2)
                    del Wm
            for name, pk, u8 in (("count_stream", False, False), ("count_stream_packed", True, False),
                                 ("count_stream_packed_u8", True, True)):
                # (u32 counts: n < 2^32; the uint8 form holds any count)
                if name in legs and (not pk or (args.kind == "dna" and m <= 32 and (u8 or N < 2 ** 32))):
                    lg[name] = stream_leg(
                        name, "count of %d x %d M patterns streamed from page-locked host memory "
                        "(%s), H2D of the next chunk overlapped with the count and the D2H of the "
                        "previous counts" % (args.stream_chunks, B // 1000000,
                                             ("2-bit packed DNA, exact uint8 counts + pairs" if u8 else
                                              "2-bit packed DNA, u32 counts") if pk else
                                             "byte strings + u64 offsets, u64 counts"),
                        idx, W, dev, sh, counts, chunks=args.stream_chunks, packed=pk, u8=u8)
            if "host_batch" in legs and counts is not None:
                # the batch handed over in host memory (PCIe in and out inside the call)
                hbuf = W.pats.cpu().numpy()
                hoffs = W.offs.cpu().numpy().astype(np.uint64)
                ht = []
                for it in range(3):
                    t1 = time.perf_counter()
                    hc = idx.count_batch(buf=hbuf, offs=hoffs)
                    ht.append(time.perf_counter() - t1)
                lg["host_batch"] = {"patterns": B, "seconds": min(ht), "patterns_per_s": B / min(ht),
                                    "h2d_bytes": int(hbuf.nbytes + hoffs.nbytes),
                                    "matches_device_batch": bool(np.array_equal(hc, counts.astype(np.uint64)))}
                del hbuf, hoffs, hc
            if "extract" in legs and args.extract_batch:
                K_, XL = args.extract_batch, 20
                g = torch.Generator(device="cpu").manual_seed(7)
                xpos = torch.randint(0, N - XL, (K_,), generator=g, dtype=torch.int64).to(dev)
                xlen = torch.full((K_,), XL, dtype=torch.int64, device=dev)
                xoff = torch.arange(0, (K_ + 1) * XL, XL, dtype=torch.int64, device=dev)
                xout = torch.empty(K_ * XL, dtype=torch.uint8, device=dev)
                xt = []
                for it in range(3):
                    torch.cuda.synchronize()
                    t1 = time.perf_counter()
                    idx.extract_device(xpos.data_ptr(), xlen.data_ptr(), xoff.data_ptr(), K_,
                                       xout.data_ptr(), sh)
                    torch.cuda.synchronize()
                    xt.append(time.perf_counter() - t1)
                want = text[(xpos.unsqueeze(1) + torch.arange(XL, device=dev)).long()].reshape(-1)
                lg["extract"] = {"queries": K_, "len": XL, "seconds": min(xt),
                                 "queries_per_s": K_ / min(xt), "bytes_per_s": K_ * XL / min(xt),
                                 "verified": bool(torch.equal(want, xout)),
                                 "method": ("copy from the text in HBM (text_.substr)" if info.text_in_hbm
                                            else "LF inversion from inverse-SA samples")}
                del xpos, xlen, xoff, xout, want

    # ---- p50 single-pattern latency (>= 1000 single-pattern calls
    #      through the C++ facade, end to end, as tools/benchmark.cpp:154-166) ----
    with LegGuard(leg_errors, "p50"):
        if rank == 0 and args.p50_calls and counts is not None:
            import ctypes as C
            hp = np.ascontiguousarray(W.pats[: args.p50_calls * m].cpu().numpy())
            nq = hp.size // m
            blib = C.CDLL(os.path.join(os.path.dirname(pkg.__file__), "libcs_bench.so"))
            fn = blib.cs_bench_facade_count_latency
            fn.restype = C.c_int
            fn.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p,
                           C.c_int]

            def facade_p50(serve):
                cnt1 = np.zeros(nq, np.uint64)
                lat = np.zeros(nq, np.float64)
                if fn(idx._h, hp.ctypes.data, m, nq, cnt1.ctypes.data, lat.ctypes.data, serve) != 0:
                    raise RuntimeError("p50 facade loop failed: " + pkg.lib().cs_fm_last_error().decode())
                assert np.array_equal(cnt1, counts[:nq].astype(np.uint64))
                return lat

            # serving mode (FMIndex::serve: a resident wave answers from a pinned mailbox)
            # is the headline p50; the one-launch-per-call path is reported beside it
            lat = facade_p50(1)
            lat_launch = facade_p50(0)
            res["p50_us"] = float(np.median(lat))
            res["p95_us"] = float(np.percentile(lat, 95))
            res["p99_us"] = float(np.percentile(lat, 99))  # as tools/benchmark.cpp:164-168
            res["max_us"] = float(np.max(lat))
            res["p50_method"] = ("cs::FMIndex::count via the C++ facade in serving mode "
                                 "(FMIndex::serve), %d calls, steady_clock" % nq)
            res["p50_launch_us"] = float(np.median(lat_launch))
            res["p95_launch_us"] = float(np.percentile(lat_launch, 95))
            res["p99_launch_us"] = float(np.percentile(lat_launch, 99))
            lat_py = []
            for q in range(min(nq, 1000)):
                b = hp[q * m:(q + 1) * m].tobytes()
                t1 = time.perf_counter()
                idx.count(b)
                lat_py.append((time.perf_counter() - t1) * 1e6)
            res["p50_python_us"] = float(np.median(lat_py))
            res["in_batch_us_per_query"] = res["ms_per_step"] * 1e3 / B

    # ---- CPU baseline: the reference's count() and locate() on host cores (rank 0, N=1) ----
    with LegGuard(leg_errors, "cpu baseline"):
        if rank == 0 and world == 1 and not args.no_cpu and counts is not None:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O  # CPU baseline / checker only
            # the process's CPU share: the affinity set, capped by OMP_NUM_THREADS where the pool
            # sets it (the GPU box: 16 per GPU; the host's core count is many times that and is
            # not ours to use) — reported with the host's count beside it
            affinity = len(os.sched_getaffinity(0))
            omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
            threads = args.cpu_threads or (min(affinity, omp) if omp else affinity)
            cpu_share = {"cores_used": threads, "host_cores": os.cpu_count(), "affinity_cores": affinity,
                         "omp_num_threads": omp or None,
                         "share": ("--cpu-threads" if args.cpu_threads else
                                   "OMP_NUM_THREADS (the pool's CPU share per GPU) within the affinity set"
                                   if omp and omp < affinity else "the whole affinity set")}
            Q = args.cpu_queries
            wide = N >= 2 ** 32  # C5: the reference's u32 tables cannot hold it
            if Q is None:
                # one pattern per thread at n >= 2^32: a faithful count() there scans 8 x 4 GB
                # bitvectors per rank (~1 min per 20-mer)
                Q = threads if wide else max(256 if N <= 200_000_000 else 32 if N <= 2_000_000_000 else 16,
                                             2 * threads)
            t1 = time.perf_counter()
            host_text = None
            try:
                d_bwt = torch.empty(N, dtype=torch.uint8, device=dev)
            except torch.OutOfMemoryError:
                # (C5: the 237-GB index, the 32-GB text and a 32-GB BWT do not fit together —
                # the text waits in host memory while the BWT comes out)
                host_text = text.cpu()
                del text
                torch.cuda.empty_cache()
                d_bwt = torch.empty(N, dtype=torch.uint8, device=dev)
            idx.bwt_device(d_bwt.data_ptr(), sh)
            bwt = d_bwt.cpu().numpy()
            del d_bwt
            if host_text is not None:
                torch.cuda.empty_cache()
                text = host_text.to(dev)
                del host_text
            ref = O.Index(bwt=bwt, nthreads=threads)
            prep_s = time.perf_counter() - t1
            sample = W.pats[: Q * m].cpu().numpy()
            soffs = np.arange(0, (Q + 1) * m, m, dtype=np.uint64)
            nt = min(threads, Q)
            Qp = min(Q, nt)  # the restatement: one pattern per thread
            t1 = time.perf_counter()
            cnt, lat = ref.count_batch(buf=sample[: Qp * m], offs=soffs[: Qp + 1], nthreads=nt,
                                       faithful=True, latencies=True)
            cpu_s = time.perf_counter() - t1
            port = {
                "value": Qp / cpu_s, "unit": "patterns/s", "cores": nt, "kind": "port",
                "sample": "first %d patterns of the batch, reference-faithful count() "
                          "(oracle/fm_oracle.c faithful=1), %d host threads" % (Qp, nt),
                "p50_us": float(np.median(lat) / 1e3), "seconds": cpu_s, "prep_s": prep_s,
                "matches_gpu": bool(np.array_equal(cnt, counts[:Qp].astype(np.uint64)))}
            port.update(cpu_share)
            res["cpu_baseline"] = port
            if O.ref_lib() is not None and not wide:
                # the genuine reference's FMIndex::count / locate (oracle/_ref/libcs_ref.so,
                # built from the reference's sources) over its own BitVector tables of the
                # same BWT, plus its bwt_ and ssa_ members for locate
                t1 = time.perf_counter()
                gref = O.RefCountIndex(ref)
                ssa = idx.ssa().astype(np.uint32)
                gref.attach_locate(bwt, ssa, args.ssa_stride)
                rprep = time.perf_counter() - t1
                t1 = time.perf_counter()
                rcnt, rlat = gref.count_batch(sample, soffs, nthreads=nt, latencies=True)
                ref_s = time.perf_counter() - t1
                res["cpu_baseline"] = {
                    "value": Q / ref_s, "unit": "patterns/s", "cores": nt, "kind": "reference",
                    "sample": "first %d patterns of the batch (%d per thread), the reference's own "
                              "FMIndex::count (src/api/fm_index.cpp:79-101, oracle/_ref/libcs_ref.so) "
                              "over its BitVector tables of the same BWT, %d host threads"
                              % (Q, Q // nt, nt),
                    "p50_us": float(np.median(rlat) / 1e3), "seconds": ref_s,
                    "prep_s": prep_s + rprep,
                    "matches_gpu": bool(np.array_equal(rcnt, counts[:Q].astype(np.uint64))), **cpu_share}
                # all host cores: the GPU pool's rules give this process 16
                # threads per GPU (OMP_NUM_THREADS; the host's other cores run other jobs), so the
                # reference's count is not timed on all of them here; its per-core rate and that
                # rate times the host's cores are reported — an upper bound for this
                # embarrassingly parallel workload, labelled as a projection, not a measurement
                per_core = Q / ref_s / nt
                res["cpu_baseline"]["per_core_value"] = per_core
                res["cpu_baseline"]["all_host_cores_projection"] = {
                    "value": per_core * (os.cpu_count() or nt), "cores": os.cpu_count(),
                    "measured": False,
                    "why": "the pool's CPU share is %d threads per GPU (OMP_NUM_THREADS); linear "
                           "scaling of the measured per-core rate" % nt}
                res["cpu_port"] = port
                # locate: one pattern per thread (a C4 locate is the count's search plus ~31
                # LF steps, each a wavelet rank with the O(n) scans)
                Ql = nt
                t1 = time.perf_counter()
                nout, lpos, llat = gref.locate_batch(sample[: Ql * m], soffs[: Ql + 1], limit=100000,
                                                     nthreads=nt)
                loc_s = time.perf_counter() - t1
                # the GPU's positions of the same patterns
                d_sp = torch.empty(Ql, dtype=torch.int64, device=dev)
                d_oo = torch.empty(Ql + 1, dtype=torch.int64, device=dev)
                gt = idx.locate_ranges_device(W.pats.data_ptr(), W.offs.data_ptr(), Ql, 100000,
                                              d_sp.data_ptr(), d_oo.data_ptr(), sh)
                d_pos = torch.empty(max(gt, 1), dtype=torch.int64, device=dev)
                idx.locate_walk_device(d_sp.data_ptr(), d_oo.data_ptr(), Ql, gt, d_pos.data_ptr(), sh)
                goo, gpos = d_oo.cpu().numpy(), d_pos[:gt].cpu().numpy()
                lok = all(nout[q] == goo[q + 1] - goo[q] and
                          lpos[q, :min(nout[q], lpos.shape[1])].tolist() ==
                          gpos[goo[q]:goo[q] + min(nout[q], lpos.shape[1])].tolist() for q in range(Ql))
                res["cpu_locate"] = {
                    "value": Ql / loc_s, "unit": "patterns/s", "cores": nt, "kind": "reference",
                    "sample": "first %d patterns of the batch (one per thread), the reference's own "
                              "FMIndex::locate (src/api/fm_index.cpp:107-157), limit 100000, row-sampled "
                              "SSA stride %d, %d host threads" % (Ql, args.ssa_stride, nt),
                    "p50_us": float(np.median(llat) / 1e3), "seconds": loc_s,
                    "positions": int(max(nout.sum(), 0)), "matches_gpu": bool(lok)}
                del gref, d_sp, d_oo, d_pos
            Qf = min(args.cpu_fast_queries, B)
            if Qf > 0:
                fs = W.pats[: Qf * m].cpu().numpy()
                foffs = np.arange(0, (Qf + 1) * m, m, dtype=np.uint64)
                t1 = time.perf_counter()
                fcnt = ref.count_batch(buf=fs, offs=foffs, nthreads=threads, faithful=False)
                fast_s = time.perf_counter() - t1
                res["cpu_fast"] = {
                    "value": Qf / fast_s, "unit": "patterns/s", "cores": threads, "kind": "port",
                    "sample": "first %d patterns of the batch, oracle count() with precomputed "
                              "totals (not the reference's cost model), %d host threads" % (Qf, threads),
                    "seconds": fast_s, "matches_gpu": bool(np.array_equal(fcnt, counts[:Qf].astype(np.uint64)))}
            del ref, bwt

    # ---- N = 1 legs on the reference's own structure: the binary wavelet matrix ----
    if idx is not None and (legs & (set(LEGS_WM) | set(LEGS_WALK) | set(LEGS_LEARNED) | set(LEGS_RDNA)
                                    | set(LEGS_FOOT))):
        del idx
        idx = None
        torch.cuda.synchronize()
    with LegGuard(leg_errors, "wavelet legs"):
        if legs & set(LEGS_WM):
            wm, bs = build_index(pkg, text, N, args.ssa_stride, local_dev,
                                 {"CS_FM_ENGINE": "wavelet", "CS_FM_FULL_SA": "0"})
            wi = wm.info()
            wwl = workload_key(args.kind, N, m, B, wi, args.queries)
            log(rank, "wavelet index built in %.1f s" % bs)
            for name, fl, what in (("wm_count", 0, "the reference's 8-level binary wavelet matrix "
                                    "(src/core/wavelet.cpp:59-96 over BitVector::rank1, bitvector.cpp:"
                                    "165-230) in 32-B rank lines: prefix table, then one rank-line pair "
                                    "per non-pure level per step"),
                                   ("wm_lf_loop", 1, "the reference's structure and its whole backward-"
                                    "search loop from C[] (fm_index.cpp:84-98): every character an "
                                    "8-level wavelet rank pair (CS_Q_NO_PREFIX)")):
                if name in legs:
                    o8 = torch.empty(B, dtype=torch.int64, device=dev)
                    lg[name], _ = count_leg(
                        name, what, wm, wi, wwl, W,
                        lambda fl=fl, o8=o8: wm.count_device_ex(W.pats.data_ptr(), W.offs.data_ptr(), B,
                                                                o8.data_ptr(), flags=fl, stream=sh),
                        fl, stream_m + 8 * B, max(3, args.steps // 8), 1, stream, sh, dev, counts,
                        lambda o8=o8: o8.cpu().numpy())
                    lg[name]["build_s"] = bs
                    del o8
            if "wm_locate_ssa" in legs:
                lg["wm_locate_ssa"] = locate_leg(
                    "wm_locate_ssa", "the reference's locate on its own structure: backward search, then the SSA walk "
                    "(fm_index.cpp:125-153) by LF over the 8-level wavelet matrix to a row with row %% "
                    "%d == 0" % args.ssa_stride, wm, wi, wwl, W, text, 0, dev, sh, reps=2)
            del wm
            torch.cuda.synchronize()
    with LegGuard(leg_errors, "walk legs"):
        if legs & set(LEGS_WALK):
            wk, bs = build_index(pkg, text, N, args.ssa_stride, local_dev, {"CS_FM_FULL_SA": "0"})
            ki = wk.info()
            log(rank, "walk-line index built in %.1f s" % bs)
            kwl = workload_key(args.kind, N, m, B, ki, args.queries) + ":walk"
            lg["locate_ssa"] = locate_leg(
                "locate_ssa", "locate without the full suffix array (the C5 layout at C4): SSA stride %d, LF walk over "
                "walk lines (symbol, occ and sample mark in one 32-B line) to the first row the "
                "reference samples or a text position marked every %d" % (args.ssa_stride, ki.position_stride),
                wk, ki, kwl, W, text, 0, dev, sh)
            lg["locate_ssa"]["build_s"] = bs
            del wk
            torch.cuda.synchronize()

    with LegGuard(leg_errors, "learned legs"):
        if legs & set(LEGS_LEARNED) and args.kind == "dna":
            lx, bs = build_index(pkg, text, N, args.ssa_stride, local_dev, {"CS_FM_ENGINE": "learned"})
            li = lx.info()
            lwl = workload_key(args.kind, N, m, B, li, args.queries)
            log(rank, "learned-lines index built in %.1f s" % bs)
            for name, fl, what in (("learned_count", 0, "the headline on learned occurrence lines (%d rows "
                                    "per 32-B line: int16 residuals against a linear model per superblock, "
                                    "src/core/bitvector_learned.cpp:114-203)" % li.line_bits),
                                   ("learned_lf_loop", 3, "the reference's whole backward-search loop over the "
                                    "learned occurrence lines (CS_Q_NO_PREFIX | CS_Q_NO_CONTEXTS)")):
                if name in legs:
                    o8 = torch.empty(B, dtype=torch.int64, device=dev)
                    lg[name], _ = count_leg(
                        name, what, lx, li, lwl, W,
                        lambda fl=fl, o8=o8: lx.count_device_ex(W.pats.data_ptr(), W.offs.data_ptr(), B,
                                                                o8.data_ptr(), flags=fl, stream=sh),
                        fl, stream_m + 8 * B, max(3, args.steps // 8), 1, stream, sh, dev, counts,
                        lambda o8=o8: o8.cpu().numpy())
                    lg[name].update({"build_s": bs, "rank_line_bytes": li.rank_bytes,
                                     "index_hbm_bytes": int(li.device_bytes)})
                    del o8
            del lx
            torch.cuda.synchronize()

    with LegGuard(leg_errors, "footprint"):
        if "footprint" in legs:
            # the throughput each rung of HBM buys: count of the headline batch (kernel time,
            # HIP events) and locate (both phases, wall) on the same text, one rung at a time
            ladder = []
            for rung, what, env in FOOT_RUNGS:
                fx, bs = build_index(pkg, text, N, args.ssa_stride, local_dev, env)
                fi = fx.info()
                nbytes = int(fi.device_bytes)
                o8 = torch.empty(B, dtype=torch.int64, device=dev)
                wall, kern_s, _ = time_launches(
                    lambda: fx.count_batch_device(W.pats.data_ptr(), W.offs.data_ptr(), B, o8.data_ptr(), sh),
                    max(3, args.steps // 8), 1, stream)
                ok = counts is None or bool(np.array_equal(o8.cpu().numpy(), counts))
                del o8
                d_sp = torch.empty(B, dtype=torch.int64, device=dev)
                d_oo = torch.empty(B + 1, dtype=torch.int64, device=dev)
                lt = []
                for it in range(2):
                    torch.cuda.synchronize()
                    t1 = time.perf_counter()
                    tot = fx.locate_ranges_device(W.pats.data_ptr(), W.offs.data_ptr(), B, 100000,
                                                  d_sp.data_ptr(), d_oo.data_ptr(), sh)
                    d_pos = torch.empty(max(tot, 1), dtype=torch.int64, device=dev)
                    fx.locate_walk_device(d_sp.data_ptr(), d_oo.data_ptr(), B, tot, d_pos.data_ptr(), sh)
                    torch.cuda.synchronize()
                    lt.append(time.perf_counter() - t1)
                    del d_pos
                del d_sp, d_oo
                ladder.append({"rung": rung, "adds": what, "index_bytes": nbytes,
                               "bytes_per_text_byte": nbytes / N, "build_s": bs,
                               "engine": engine_name(fi), "prefix_k": fi.prefix_k,
                               "count_patterns_per_s": B / kern_s, "count_kernel_ms": kern_s * 1e3,
                               "count_matches_headline": ok,
                               "locate_patterns_per_s": B / min(lt), "locate_ms": min(lt) * 1e3})
                log(rank, "footprint %s: %.1f GB, count %.3g/s, locate %.3g/s" % (
                    rung, nbytes / 1e9, B / kern_s, B / min(lt)))
                del fx
                torch.cuda.synchronize()
            lg["footprint"] = {"what": "the same text and batch indexed with the optional structures "
                                       "added one at a time (HBM footprint vs throughput)",
                               "rungs": ladder}

    with LegGuard(leg_errors, "budget"):
        if "budget" in legs:
            # the same text under an HBM budget (CS_FM_HBM_BUDGET): the engine adds its optional
            # structures in build order while the index fits
            full_b = lg.get("footprint", {}).get("rungs", [{}])[-1].get("index_bytes")
            if not full_b:
                fx, _ = build_index(pkg, text, N, args.ssa_stride, local_dev)
                full_b = int(fx.info().device_bytes)
                del fx
            rows = []
            for fr in BUDGET_FRACS:
                budget = int(full_b * fr)
                fx, bs = build_index(pkg, text, N, args.ssa_stride, local_dev,
                                     {"CS_FM_HBM_BUDGET": str(budget)})
                fi = fx.info()
                nbytes = int(fi.device_bytes)
                o8 = torch.empty(B, dtype=torch.int64, device=dev)
                wall, kern_s, _ = time_launches(
                    lambda: fx.count_batch_device(W.pats.data_ptr(), W.offs.data_ptr(), B, o8.data_ptr(), sh),
                    max(3, args.steps // 8), 1, stream)
                ok = counts is None or bool(np.array_equal(o8.cpu().numpy(), counts))
                del o8
                rows.append({"budget_bytes": budget, "index_bytes": nbytes, "build_s": bs,
                             "prefix_k": fi.prefix_k, "left_contexts": bool(fi.context_bytes),
                             "record_bytes": fi.record_bytes, "walk_lines": bool(fi.walk_bytes),
                             "full_sa": bool(fi.full_sa_bytes), "text_in_hbm": bool(fi.text_in_hbm),
                             "count_patterns_per_s": B / kern_s, "count_matches_headline": ok})
                log(rank, "budget %.1f GB: %.1f GB, count %.3g/s" % (budget / 1e9, nbytes / 1e9, B / kern_s))
                del fx
                torch.cuda.synchronize()
            lg["budget"] = {"what": "CS_FM_HBM_BUDGET at fractions of the default footprint (%d B)" % full_b,
                            "rows": rows}

    with LegGuard(leg_errors, "repetitive-DNA legs"):
        # (a second text and index of the headline's size: C4-sized configs only — at C5 the
        # two 32-GB texts and the index do not fit beside each other)
        if legs & set(LEGS_RDNA) and args.kind == "dna" and N < 2 ** 32:
            # repetitive DNA: copies of a 2^20-base seed with ~0.75 % substitutions, so a
            # text 20-mer occurs in most of the ~3800 copies: ranges thousands of rows wide
            # step through the rank structure instead of ending in a context record
            rtext = torch.empty(N + 16, dtype=torch.uint8, device=dev)
            pkg.synth_text_device("rdna", 42, L, rtext.data_ptr(), sh)
            torch.cuda.synchronize()
            rx, bs = build_index(pkg, rtext, N, args.ssa_stride, local_dev)
            ri = rx.info()
            rwl = workload_key("rdna", N, m, B, ri, args.queries)
            log(rank, "repetitive-DNA index built in %.1f s" % bs)
            RW = Workload(pkg, rtext, N, m, lo, B, args.kind, args.queries, dev, sh)
            o8 = torch.empty(B, dtype=torch.int64, device=dev)
            if "count_rdna" in legs:
                r, got = count_leg(
                    "count_rdna", "Q_text 20-mers of a repetitive DNA text of the same size (copies of a "
                    "2^20-base seed, ~0.75 %% substitutions; cs_synth_text_device kind 2) through the "
                    "headline engine", rx, ri, rwl, RW,
                    lambda: rx.count_batch_device(RW.pats.data_ptr(), RW.offs.data_ptr(), B, o8.data_ptr(), sh),
                    0, stream_m + 8 * B, max(3, args.steps // 4), 1, stream, sh, dev, None,
                    lambda: o8.cpu().numpy())
                # the search paths taken, from the per-query bytes of the measurement twin:
                # one 16-B context record alone, or more reads (context sectors, rank steps)
                qb = torch.empty(B, dtype=torch.int64, device=dev)
                rx.count_bytes_device(RW.pats.data_ptr(), RW.offs.data_ptr(), B, qb.data_ptr(), sh)
                eb = ri.prefix_bytes // (ri.prefix_sigma ** ri.prefix_k) if ri.prefix_k else 0
                r.update({"build_s": bs, "found_frac": float((got >= 1).mean()),
                          "count_mean": float(got.mean()), "count_p50": float(np.median(got)),
                          "count_p99": float(np.percentile(got, 99)), "count_max": int(got.max()),
                          "record_only_frac": float((qb == eb).float().mean().item()),
                          "fallback_frac": float((qb > eb).float().mean().item())})
                del qb
                lg["count_rdna"] = r
            if "locate_rdna" in legs:
                # 1/125 of the batch: ~3,300 positions per pattern at limit 100000
                LB = max(1, B // 125)
                LW = Workload.__new__(Workload)
                LW.m, LW.B, LW.pats, LW.offs = m, LB, RW.pats[: LB * m], RW.offs[: LB + 1]
                lg["locate_rdna"] = locate_leg(
                    "locate_rdna", "locate (limit 100000) of %d repetitive-DNA 20-mers: thousands of "
                    "positions per pattern from the full suffix array" % LB, rx, ri, rwl, LW, rtext, 0,
                    dev, sh, reps=2)
            del rx, RW, o8, rtext
            torch.cuda.synchronize()

    if rank == 0:
        if args.only:
            res = {"only": args.only, "workload_key": wl if need_main else None,
                   **({"count": res.get("roofline")} if args.only == "count" else {}),
                   "legs": lg}
        if leg_errors:
            res["leg_errors"] = leg_errors
        if lg and not args.only:
            # locate at the top level: the one-call form (cs_fm_locate_device), else the
            # two phases
            if "locate_one" in lg or "locate" in lg:
                res["locate"] = lg.get("locate_one") or lg["locate"]
            res["legs"] = lg
        legs_file = None
        if args.legs_out != "none" and not args.only:
            legs_file = args.legs_out or os.path.join(
                "gpurun_out", "bench_full_n%d_%s.json" % (world, time.strftime("%Y%m%d_%H%M%S")))
            try:
                path = legs_file if os.path.isabs(legs_file) else os.path.join(ROOT, legs_file)
                os.makedirs(os.path.dirname(path), exist_ok=True)
                with open(path, "w") as f:
                    json.dump(res, f)
            except OSError as e:
                log(rank, "could not write %s: %s" % (legs_file, e))
                legs_file = None
        if not args.only:
            # the full result (every leg) on stderr as well, one line
            print("[bench] full result: " + json.dumps(res), file=sys.stderr, flush=True)
        print(compact_line(res, legs_file), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
