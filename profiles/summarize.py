#!/usr/bin/env python3
"""summarize.py <prof_dir> <tag> — condense rocprofv3 CSV output of
profile_count.sh into <prof_dir>/summary.json:

  kernels: per kernel name, dispatch count and mean/min/max duration (ns) from
           the --kernel-trace --stats pass;
  pmc:     per hot kernel, mean FETCH_SIZE (KB per dispatch, as reported) and the
           L2 hit rate TCC_HIT/(TCC_HIT+TCC_MISS) from their own passes.
  bench:   the bench JSON line each pass printed (the un-profiled numbers are in
           BENCH_rNN.json; profiled passes run slower, MI355X_MICROARCH 'DVFS
           give-back' item 2).
FETCH_SIZE is reported raw in `pmc`; pmc_count.json converts it to HBM bytes with
the request mix of the count kernel (see the correction note written there).
"""
import csv
import glob
import json
import os
import statistics
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def _ctx_is_loc(name):
    """k_count_ctx<E, U, kLoc, ...>: its third template argument (demangled, or the mangled
    ...EELi<U>ELb<kLoc>E form)."""
    import re
    m = re.search(r"k_count_ctx<[^,]+,\s*\d+,\s*(true|false)", name)
    if m:
        return m.group(1) == "true"
    m = re.search(r"k_count_ctxI.*?EELi\dELb([01])E", name)
    return bool(m and m.group(1) == "1")


def short(name):
    if "k_count_ctx" in name:  # count, or locate (phase 1 / the one-call search)
        return "k_count_ctx_loc" if _ctx_is_loc(name) else "k_count_ctx"
    for k in ("k_count_bytes", "k_count_one", "k_count_long", "k_count_list", "k_locate_long",
              "k_locate_list", "k_locate_emit_wide", "k_locate_emit", "k_scan_tiles", "k_count_qctx",
              "k_count_ctx", "k_count", "k_build_lctx", "k_walk_lines", "k_walk_pack",
              "k_walk_base", "k_walk_samples", "k_walk", "k_occ_pack", "k_occ_base", "k_locate_ranges", "k_expand_rows", "k_lf", "k_bwt_ssa", "k_bwt",
              "k_build_ptab", "k_locate_sa_wide", "k_locate_sa", "k_extract_text", "k_extract",
              "k_fill_records16", "k_fill_records_q", "k_fill_records",
              "k_partition", "k_pack_level", "k_init_keys", "k_double_keys", "k_heads",
              "k_scatter_rank", "k_bwt_ssa", "k_hist", "k_text", "k_patterns", "k_indep", "k_chain"):
        if k in name:
            return k
    return name[:60]


def main():
    d, tag = sys.argv[1], sys.argv[2]
    res = {"tag": tag, "kernels": {}, "pmc": {}, "bench": {}}
    kt = rows(os.path.join(d, "trace", "**", "*kernel_trace.csv"))
    by = {}
    for r in kt:
        n = short(r.get("Kernel_Name", ""))
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        by.setdefault(n, []).append(dur)
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        # round 5: the median over the dispatches is the figure to set beside bench.py's
        # roofline (itself a median over its timed launches) — a slow first dispatch (cold
        # TLB / caches) moves the mean, not the median
        res["kernels"][n] = {"dispatches": len(v), "median_ns": statistics.median(v),
                             "mean_ns": statistics.mean(v), "min_ns": min(v),
                             "max_ns": max(v), "total_ns": sum(v),
                             "median_after_first_ns": statistics.median(v[1:]) if len(v) > 1 else None}
    for sub, names in (("pmc_fetch", ["FETCH_SIZE"]), ("pmc_l2", ["TCC_HIT_sum", "TCC_MISS_sum"])):
        for r in rows(os.path.join(d, sub, "**", "*counter_collection.csv")):
            n = short(r.get("Kernel_Name", ""))
            c = r.get("Counter_Name")
            if c in names:
                res["pmc"].setdefault(n, {}).setdefault(c, []).append(float(r["Counter_Value"]))
    for n, cs in res["pmc"].items():
        for c, v in list(cs.items()):
            cs[c] = statistics.mean(v)
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            tot = cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"]
            cs["l2_hit_rate"] = cs["TCC_HIT_sum"] / tot if tot else None
    for f in ("bench_trace.json", "bench_fetch.json", "bench_l2.json"):
        p = os.path.join(d, f)
        if os.path.exists(p):
            try:
                res["bench"][f] = json.loads(open(p).read().strip().splitlines()[-1])
            except Exception:
                pass
    # stats CSV from pass 1 (copied next to the summary)
    st = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if st:
        res["kernel_stats_csv"] = os.path.relpath(st[0], d)
    with open(os.path.join(d, "summary.json"), "w") as f:
        json.dump(res, f, indent=1)
    # pmc_count.json for bench.py's roofline.traffic (copy into profiles/ to use)
    b = res["bench"].get("bench_trace.json") or {}
    kname = "k_count_ctx" if "FETCH_SIZE" in res["pmc"].get("k_count_ctx", {}) else "k_count"
    kc = res["pmc"].get(kname, {})
    if b and "FETCH_SIZE" in kc:
        # FETCH_SIZE = TCC_EA0_RDREQ x 64 B.  Requests of this kernel: random 32-B
        # reads (rank lines, context sectors, table entries: one request each, tallied
        # at 64 B — profiles/microbench/gather_bench calibration) and the coalesced
        # stream of patterns + offsets (128-B requests tallied at 64 B, the guide's
        # gfx950 x2).  bytes = stream + (requests - stream / 128) x 32.
        cfg = b.get("config", {})
        B, m = cfg.get("batch_per_gpu", 0), cfg.get("m", 0)
        stream = B * m + (B + 1) * 8
        req = kc["FETCH_SIZE"] * 1024 / 64
        pc = {"workload": cfg.get("workload_key"), "kernel": kname,
              "fetch_size_kb_per_launch": kc["FETCH_SIZE"],
              "read_requests_per_launch": req,
              "stream_bytes_per_launch": stream,
              "hbm_bytes_per_launch": stream + max(req - stream / 128, 0) * 32,
              "correction": "FETCH_SIZE/64 B = read requests; the pattern/offset stream "
                            "(B*m + 8(B+1) bytes, 128-B requests) counted at its byte size, "
                            "every other request a random 32-B read (calibrated with "
                            "profiles/microbench/gather_bench: 1 request per random 32-B "
                            "read, FETCH_SIZE = 64 B per read)",
              "l2_hit_rate": kc.get("l2_hit_rate"),
              "tcc_miss_per_launch": kc.get("TCC_MISS_sum"),
              "kernel_mean_ns_profiled": res["kernels"].get(kname, {}).get("mean_ns"),
              "tag": tag}
        with open(os.path.join(d, "pmc_count.json"), "w") as f:
            json.dump(pc, f, indent=1)
    print(json.dumps({"kernels": {k: v["mean_ns"] for k, v in res["kernels"].items()},
                      "pmc": res["pmc"]}, indent=1))


if __name__ == "__main__":
    main()
