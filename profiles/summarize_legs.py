#!/usr/bin/env python3
"""summarize_legs.py <prof_dir> <tag> — condense profile_legs.sh's rocprofv3 output.

For every leg directory <prof_dir>/<leg>/: the per-kernel durations of the trace pass,
the mean FETCH_SIZE and L2 hit rate of each profiled kernel, and the leg's own kernel
(the count kernel of a count leg, the phase-2 kernel of a locate leg).  Writes
<prof_dir>/stats.json and <prof_dir>/pmc_legs.json — the file bench.py reads as
profiles/pmc_legs.json:

  "<workload key>|<leg>": {kernel, fetch_size_kb_per_launch, read_requests_per_launch,
                           stream_read_bytes_per_launch, hbm_bytes_per_launch, ...}

HBM bytes from FETCH_SIZE (= TCC_EA0_RDREQ x 64 B on gfx950, MI355X_MICROARCH.md): the
kernel's streamed reads (coalesced 128-B requests, tallied at 64 B — the guide's x2)
count at their byte size, every other request is one random 32-B DRAM read (calibrated
with profiles/microbench/gather_bench: one request per random read of 16-32 B, tallied
at 64 B; profiles/r01/fetch_calibration.txt).
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from srchash import kernel_src_hash  # noqa: E402  (the tree that was profiled)

ONE_CALL = ("k_count_ctx_onepass", "k_count_ctx_onepass_skiplong", "k_count_qctx_onepass", "k_locate_one_gen",
            "k_locate_long", "k_locate_list",
            "k_locate_emit", "k_locate_emit_wide", "k_locate_walks", "k_scan_chained", "k_scan_tiles")
# the kernel that carries each leg's work
LEG_KERNEL = {"count": "count", "count_u32": "count", "count_packed": "count",
              "count_table_steps": "count", "count_lf_loop": "count", "count_m32": "count",
              "count_m64": "count", "count_m64_steps": "count", "count_m150": "count",
              "count_fixed": "count", "wm_count": "count", "count_m150_staged": "count",
              "count_m64_long": "count", "count_m150_long": "count",
              "wm_lf_loop": "count", "learned_count": "count", "learned_lf_loop": "count",
              "count_unif": "count",
              "locate": ("k_locate_sa", "k_locate_sa_wide", "k_walk_fused", "k_walk_fused_wide",
                         "k_walk_lines", "k_walk_short"),
              "locate_ssa_rows": "k_walk", "wm_locate_ssa": "k_walk",
              "locate_ssa": ("k_walk_fused", "k_walk_fused_wide"), "count_rdna": "count",
              "locate_rdna": ("k_locate_sa", "k_locate_sa_wide"),
              # the one-call locate: every kernel of the call (search, long-pattern search and
              # its list, positions), summed per launch
              "locate_one": ONE_CALL, "locate_m64": ONE_CALL, "locate_m150": ONE_CALL}

# legs whose phase-2 reads are contiguous runs of the suffix array, not random rows
LEG_STREAMED = {"locate_rdna"}
# bytes the HBM moves for one random read request (round 4; rounds 1-3 assumed 32)
DRAM_ACCESS = 64


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def short(name):
    """Readable kernel name: k_count_ctx (count) / k_count_ctx_loc (locate phase 1) with
    the template's U, packed flag and count width; the others by their base name."""
    m = re.search(r"k_count_ctx<[^,]*?(\w+E?), (\d), (true|false), (true|false), (\d)"
                  r"(?:, (true|false))?(?:, (true|false))?(?:, (true|false))?(?:, (true|false))?(?:, (\d))?>", name)
    if m:
        eng, u, loc, packed, w, nobar, one, skip, rng, pos = m.groups()
        if one == "true":  # the one-call locate's search (skiplong: under long-pattern routing)
            return "k_count_ctx_onepass%s" % ("_skiplong" if skip == "true" else "")
        if loc == "true":
            return "k_count_ctx_loc"
        return "k_count_ctx%s%s_w%s" % ("_packed" if packed == "true" else "",
                                         "_skiplong" if skip == "true" else "", w)
    m = re.search(r"k_count_long<(\d), (true|false)(?:, (true|false))?(?:, \d+)?(?:, (true|false))?(?:, \d+)?>",
                  name)
    if m:  # the third argument: the measurement twin (kBytes); the last (round 6) kWalk
        return "k_count_long%s%s" % ("_ptext" if m.group(2) == "true" else "_btext",
                                     "_bytes" if m.group(3) == "true" else "")
    m = re.search(r"k_count_list<(\d)(?:, (true|false))?>", name)
    if m:
        return "k_count_list_bytes" if m.group(2) == "true" else "k_count_list"
    m = re.search(r"k_count_qctx<(\d), (\d)(?:, (true|false))?>", name)
    if m:  # (round 6) the third argument: the one-call locate's search (kOne)
        return "k_count_qctx_onepass" if m.group(3) == "true" else "k_count_qctx_w%s" % m.group(2)
    m = re.search(r"k_count<[^,]*?(\w+)(<\w+>)?, (true|false)>", name)
    if m:
        return "k_count_packed" if m.group(3) == "true" else "k_count"
    for k in ("k_walk_samples", "k_walk_pack", "k_walk_base"):  # index build
        if k in name:
            return k
    for k in ("k_count_bytes", "k_count_one", "k_count", "k_walk_short", "k_walk_lines", "k_walk_fused_wide",
              "k_walk_fused", "k_walk", "k_locate_walks", "k_scan_chained", "k_scan_tiles",
              "k_locate_long", "k_locate_list", "k_locate_emit_wide", "k_locate_emit", "k_locate_one_gen",
              "k_locate_ranges", "k_locate_sa_wide", "k_locate_sa", "k_expand_rows", "k_pack_wire"):
        if k in name:
            return k
    return name[:48]


def last_json(path):
    try:
        return json.loads(open(path).read().strip().splitlines()[-1])
    except Exception:
        return None


def main():
    d, tag = sys.argv[1], sys.argv[2]
    stats, pmc_legs = {"tag": tag, "legs": {}}, {}
    for ld in sorted(glob.glob(os.path.join(d, "*", ""))):
        leg = os.path.basename(os.path.dirname(ld))
        res = {"kernels": {}, "pmc": {}}
        for r in rows(os.path.join(ld, "trace", "**", "*kernel_trace.csv")):
            n = short(r.get("Kernel_Name", ""))
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            res["kernels"].setdefault(n, []).append(dur)
        # (round 5: the median beside the mean — bench.py's roofline time is a median of its
        # timed launches, and the first, cold launch moves a mean)
        res["kernels"] = {n: {"dispatches": len(v), "median_ns": statistics.median(v),
                              "mean_ns": statistics.mean(v), "min_ns": min(v), "total_ns": sum(v)}
                          for n, v in sorted(res["kernels"].items(), key=lambda kv: -sum(kv[1]))}
        for sub, names in (("pmc_fetch", ["FETCH_SIZE"]), ("pmc_l2", ["TCC_HIT_sum", "TCC_MISS_sum"])):
            for r in rows(os.path.join(ld, sub, "**", "*counter_collection.csv")):
                n = short(r.get("Kernel_Name", ""))
                if r.get("Counter_Name") in names:
                    res["pmc"].setdefault(n, {}).setdefault(r["Counter_Name"], []).append(
                        float(r["Counter_Value"]))
        for n, cs in res["pmc"].items():
            for c, v in list(cs.items()):
                cs[c] = statistics.mean(v)
            if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
                tot = cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"]
                cs["l2_hit_rate"] = cs["TCC_HIT_sum"] / tot if tot else None
        b = last_json(os.path.join(ld, "bench_trace.json")) or {}
        res["bench"] = b
        # the leg's kernel and its streamed reads
        want = LEG_KERNEL.get(leg, "count")
        if want == "count":
            cands = [n for n in res["pmc"] if n.startswith("k_count_ctx_") or n.startswith("k_count_qctx")
                     or n == "k_count" or (n.startswith("k_count_long") and not n.endswith("_bytes"))]
        else:  # the phase-2 kernel that ran longest (a lane per pattern, or a block per wide range)
            want = (want,) if isinstance(want, str) else want
            cands = [n for n in res["pmc"] if n in want]
        # the timed launches: the candidate dispatched most often (a routed leg's first, warm-up
        # launch runs the staged kernel once), then the longest in total
        kname = max(cands, key=lambda n: (res["kernels"].get(n, {}).get("dispatches", 0),
                                          res["kernels"].get(n, {}).get("total_ns", 0))) if cands else None
        # a routed long-pattern count runs as k_count_ctx (skipping the long patterns),
        # k_count_long and k_count_list: the leg's launch is their sum
        group = [kname]
        if want is ONE_CALL:  # routed (the long-pattern search ran): its kernels, else the plain call's
            routed = "k_locate_long" in res["kernels"]
            group = sorted(n for n in cands if n in res["kernels"] and
                           (n != "k_count_ctx_onepass" if routed else n != "k_count_ctx_onepass_skiplong"))
        elif kname and (kname.startswith("k_count_long") or "skiplong" in kname):
            # a routed count (round 5: every device batch): the staged kernel, the list kernel
            # (long patterns and listed general searches) and k_count_list
            group += [n for n in res["pmc"] if n == "k_count_list" or
                      (n.startswith("k_count_long") and not n.endswith("_bytes")) or
                      (n.startswith("k_count_ctx_") and "skiplong" in n)]
            group = sorted(set(group))
        lo = (b.get("legs") or {}).get(leg) or {}
        if leg == "count":
            stream_rd = (b.get("count") or {}).get("stream_read_bytes_per_launch")
        elif "roofline" in lo:
            stream_rd = lo["roofline"].get("stream_read_bytes_per_launch")
        else:
            stream_rd = lo.get("phase2_stream_read_bytes")
        if want is ONE_CALL and stream_rd is not None and lo.get("patterns"):
            # the emit kernel's read of the records (round 5: no count beside a stashed position)
            stream_rd += 8 * lo["patterns"]
        wl = lo.get("workload_key") or b.get("workload_key")  # the leg's own index
        kc = res["pmc"].get(kname, {}) if kname else {}
        if len(group) > 1:  # sums over the group (per launch of each)
            kc = {"FETCH_SIZE": sum(res["pmc"].get(n, {}).get("FETCH_SIZE", 0) for n in group),
                  "l2_hit_rate": kc.get("l2_hit_rate")}
        if kname and "FETCH_SIZE" in kc and stream_rd is not None:
            req = kc["FETCH_SIZE"] * 1024 / 64
            # a leg whose kernel streams (thousands of contiguous SA rows per range): every
            # request is a 128-B streaming read tallied at 64 B (the guide's x2)
            # the rest one 64-B DRAM request per random read: TCC_EA0_RDREQ_32B_sum is 0
            # for the count kernels (profiles/r04/pmc_probe_count_packed.json: 13.47 M
            # requests per 12.5 M packed patterns, all of 64 B; FETCH_SIZE = requests x 64 B)
            hbm = (req * 128 if leg in LEG_STREAMED
                   else stream_rd + max(req - stream_rd / 128, 0) * DRAM_ACCESS)
            e = {"leg": leg, "kernel": "+".join(group) if len(group) > 1 else kname,
                 "fetch_size_kb_per_launch": kc["FETCH_SIZE"],
                 "read_requests_per_launch": req, "stream_read_bytes_per_launch": stream_rd,
                 "hbm_bytes_per_launch": hbm,
                 "l2_hit_rate": kc.get("l2_hit_rate"),
                 "kernel_mean_ns_profiled": sum(res["kernels"].get(n, {}).get("mean_ns", 0) for n in group),
                 "kernel_median_ns_profiled": sum(res["kernels"].get(n, {}).get("median_ns", 0) for n in group),
                 "dispatches_profiled": res["kernels"].get(kname, {}).get("dispatches"),
                 "tag": tag, "src_hash": kernel_src_hash()}
            e["workload"] = wl
            pmc_legs["%s|%s" % (wl, leg)] = e
            res["traffic"] = e
        stats["legs"][leg] = res
    with open(os.path.join(d, "stats.json"), "w") as f:
        json.dump(stats, f, indent=1)
    with open(os.path.join(d, "pmc_legs.json"), "w") as f:
        json.dump(pmc_legs, f, indent=1)
    print(json.dumps({k: {"kernel": v["kernel"], "hbm_bytes_per_launch": v["hbm_bytes_per_launch"],
                          "l2": v["l2_hit_rate"]} for k, v in pmc_legs.items()}, indent=1))


if __name__ == "__main__":
    main()
