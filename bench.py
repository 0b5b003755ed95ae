#!/usr/bin/env python3
"""bench.py — batched FM-index count() on MI355X (BASELINE.json metric).

Workload (default = BASELINE.json configs[3], "C4", the config the metric is
quoted on; it fits one GPU): 4 GB synthetic DNA text (n = 4e9 incl. the '$'
terminator, SURVEY.md §8(d): splitmix64 seed 42), Q_text 20-mers (substrings at
splitmix64(4242) positions).  One step = one batched count() launch over a batch
of --batch patterns per GPU, inputs resident in HBM.  Multi-GPU: one process per
GPU, index replicated (built per GPU), query stream sharded in contiguous ranges
(weak scaling: --batch per GPU).  Queries are independent, so the timed step has
no data-path collective: each rank's counts stay with its shard (barrier + max
over ranks around the K steps).  --gather adds SURVEY §8(e)'s gather of the
counts to rank 0 over RCCL, double-buffered behind the next step's count.

Extra fields on the JSON line:
  roofline     the count kernel against HBM: achieved = algorithmic bytes per
               launch / mean kernel time (HIP events on the launch stream).
               Algorithmic bytes = the random reads the search needs (prefix-table
               entry, one 32-B line per rank step, the 32-B context sector(s);
               counted per query by cs_fm_count_bytes_device) + the stream every
               launch moves (patterns, offsets, counts).  traffic = HBM bytes per
               launch from the committed rocprofv3 PMC summary for this workload.
  cpu_baseline the reference's own FMIndex::count (oracle/_ref/libcs_ref.so, built
               from its sources; kind "reference"), else the oracle's
               reference-faithful count() (kind "port"; O(n) count_ones scans, as
               src/core/bitvector.cpp:168-170), on a bounded sample of the same
               batch, rank 0, N=1 only, all host threads.
  p50_us       median end-to-end latency of single-pattern cs::FMIndex::count() calls
               through the C++ facade (host pattern in, count out), as
               tools/benchmark.cpp:154-166, with the index in serving mode (a resident
               wave answers from a pinned mailbox); p50_launch_us: the same calls with
               one kernel launch each.
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


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


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
                    help="patterns timed on the CPU (default SURVEY §8(d): 256 at C2-size texts, "
                         "32 at C3, 16 at C4 and above)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--p50-calls", type=int, default=1000)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--locate-batch", type=int, default=12_500_000,
                    help="patterns of the batch timed through locate() (N=1 only; 0 = skip)")
    ap.add_argument("--queries", default="text", choices=["text", "unif"],
                    help="Q_text (substrings of the text, the headline) or Q_unif (uniform random)")
    ap.add_argument("--cpu-fast-queries", type=int, default=1_000_000,
                    help="patterns timed through the oracle's fast (precomputed) count, all threads")
    ap.add_argument("--extract-batch", type=int, default=1_000_000,
                    help="random 20-byte extracts timed on the device (N=1 only; 0 = skip)")
    ap.add_argument("--host-batch", type=int, default=1,
                    help="also time the batch handed over in host memory (PCIe-inclusive; 0 = skip)")
    ap.add_argument("--replicate", default="build", choices=["build", "broadcast"],
                    help="N > 1: every rank builds its replica, or rank 0 builds and broadcasts "
                         "the device image (RCCL)")
    ap.add_argument("--gather", action="store_true",
                    help="gather every step's counts to rank 0 (RCCL), overlapped with the next count")
    ap.add_argument("--prefix-k", type=int, default=None,
                    help="prefix-table depth override (0 = off; default automatic)")
    args = ap.parse_args()
    if args.prefix_k is not None:
        os.environ["CS_FM_PREFIX_K"] = str(args.prefix_k)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    local_dev = local % max(ndev, 1)  # identity on an N-GPU node; lets a 1-GPU box rehearse N ranks
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
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
    if args.replicate == "broadcast" and world > 1:
        # rank 0 builds; the device image goes to every rank (shard.replicate_index)
        idx = (pkg.FMIndex.build_from_device_text(text.data_ptr(), N,
                                                  pkg.BuildParams(ssa_stride=args.ssa_stride),
                                                  device=local_dev) if rank == 0 else None)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        idx = shard.replicate_index(pkg, idx, 0, rank, world, dev)
        replicate_s = time.perf_counter() - t1
    else:
        idx = pkg.FMIndex.build_from_device_text(text.data_ptr(), N,
                                                 pkg.BuildParams(ssa_stride=args.ssa_stride),
                                                 device=local_dev)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    info = idx.info()
    log(rank, "index built: n=%d in %.1f s, rank lines %.2f GB" % (N, build_s, info.rank_bytes / 1e9))

    # ---- this rank's query shard (contiguous slice of the Q_text stream) ----
    B, m = args.batch, args.m
    total = B * world  # weak scaling: B patterns per GPU
    lo, hi = shard.shard_range(total, rank, world)
    assert hi - lo == B
    pats = torch.empty(B * m, dtype=torch.uint8, device=dev)
    offs = torch.empty(B + 1, dtype=torch.int64, device=dev)
    if args.queries == "text":
        pkg.synth_patterns_device(text.data_ptr(), N, m, lo, B, 4242, pats.data_ptr(),
                                  offs.data_ptr(), sh)
    else:  # SURVEY §8(d) secondary batch Q_unif
        pkg.synth_random_patterns_device(args.kind, m, lo, B, 4242, pats.data_ptr(),
                                         offs.data_ptr(), sh)
    # counts land in double-buffered shards; with --gather (N > 1) the gather of step
    # k to rank 0 overlaps the count of step k+1 (shard.PipelinedGather), otherwise
    # each rank keeps its shard's counts (no collective in the data path)
    coll = args.gather and world > 1
    pg = shard.PipelinedGather(B, world if coll else 1, rank if coll else 0, torch.int64, dev)

    # algorithmic bytes per launch, counted by the engine's measurement twin of the
    # count kernel (cs_fm_count_bytes_device): per backward-search step, the distinct
    # lines its rank pair (sp, ep) needs (one 32-B occurrence line, or one rank line
    # per non-pure wavelet level; sp and ep in the same line count once) times the
    # line size, plus the 8-B (16-B wide) prefix-table entry that replaces the first
    # k steps.
    line_bytes = info.line_bytes
    qbytes = torch.empty(B, dtype=torch.int64, device=dev)
    idx.count_bytes_device(pats.data_ptr(), offs.data_ptr(), B, qbytes.data_ptr(), sh)
    alg_random = int(qbytes.sum().item())
    # plus the streamed bytes every launch must move: the patterns, their offsets and
    # the counts written back
    alg_stream = B * m + (B + 1) * 8 + B * 8
    alg_bytes = alg_random + alg_stream
    del qbytes
    P2 = pats.view(B, m).long()
    K = info.prefix_k
    table_frac = 0.0
    if K and m >= K:
        code = torch.tensor(list(info.prefix_code), dtype=torch.int64, device=dev)
        table_frac = float((code[P2[:, m - K:]] != 255).all(dim=1).float().mean().item())
    del P2
    torch.cuda.synchronize()

    for k in range(args.warmup):
        o = pg.buffer(k)
        idx.count_batch_device(pats.data_ptr(), offs.data_ptr(), B, o.data_ptr(), sh)
        pg.submit(k)
    pg.finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        o = pg.buffer(k)
        evs[k][0].record(stream)
        idx.count_batch_device(pats.data_ptr(), offs.data_ptr(), B, o.data_ptr(), sh)
        evs[k][1].record(stream)
        pg.submit(k)
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
    # DRAM accesses per launch (each distinct line and each table entry is one random
    # access) against the measured random-access ceiling of MI355X:
    # profiles/microbench/gather_bench.hip, 8..32-B random reads over a 4 GB table run
    # at 49-52 G accesses/s (profiles/r01/gather_bench*.txt)
    eb = info.prefix_bytes // (info.prefix_sigma ** K) if K else 0
    hits = int(round(B * table_frac)) if K else 0
    accesses = (alg_random - eb * hits) / info.line_bytes + hits
    total_units = B * world * args.steps
    value = total_units / elapsed
    kern_avg_s = statistics.mean(kern_ms) / 1e3
    achieved = alg_bytes / kern_avg_s / 1e9
    out = pg.local[(args.steps - 1) % pg.depth]
    counts = out.cpu().numpy()
    found = int((counts >= 1).sum())

    res = None
    if rank == 0:
        traffic = None
        prof = os.path.join(ROOT, "profiles", "pmc_count.json")
        engine = {1: "occ", 2: "qwm", 3: "locc"}.get(info.engine, "wm%d" % info.line_bytes)
        wl = "%s:%d:m%d:b%d:%s:k%d" % (args.kind, N, m, B, engine, info.prefix_k)
        if info.context_q:
            wl += ":ctx%d" % info.context_q
        if info.record_bytes:
            wl += ":rec%d" % info.record_bytes  # context records (32-/16-B prefix-table entries)
        if args.queries != "text":
            wl += ":" + args.queries
        if os.path.exists(prof):
            pj = json.load(open(prof))
            if pj.get("workload") == wl:
                traffic = pj.get("hbm_bytes_per_launch")
        res = {
            "metric": METRIC,
            "value": value,
            "unit": "patterns/s",
            "n_gpus": world,
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
                       "collective": "gather of counts to rank 0 (%s), overlapped"
                       % ("RCCL" if args.dist_backend == "nccl" else args.dist_backend) if coll
                       else "none (independent query shards)",
                       "engine": ("%s + left contexts (q=%d)%s" % (
                                  "learned occurrence lines" if info.engine == 3 else "occurrence lines",
                                  info.context_q,
                                  " + %d-B context records" % info.record_bytes if info.record_bytes
                                  else "")) if info.engine in (1, 3) else
                       "quaternary wavelet matrix (%d levels of occurrence lines)" % info.levels
                       if info.engine == 2 else
                       "wavelet matrix (%d-B rank lines)" % info.line_bytes},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "alg_bytes_per_launch": alg_bytes, "alg_random_bytes_per_launch": alg_random,
                         "alg_stream_bytes_per_launch": alg_stream, "line_bytes": line_bytes,
                         "prefix_k": K, "prefix_table_hit_frac": table_frac,
                         "context_q": info.context_q,
                         "alg_bytes_per_query": alg_bytes / B,
                         # SURVEY.md §8(d)'s per-query figure for the reference's
                         # structure (64 B x 8 levels x 2 ranks x (m-1) steps), for
                         # comparison only: this engine reads alg_bytes_per_query
                         "survey_alg_bytes_per_query": 64 * 8 * 2 * (m - 1),
                         "survey_equivalent_GBs": 64 * 8 * 2 * (m - 1) * B / kern_avg_s / 1e9,
                         "random_accesses_per_launch": accesses,
                         "random_accesses_per_s": accesses / kern_avg_s,
                         "random_access_ceiling_per_s": 5.0e10,
                         "frac_of_random_access_ceiling": accesses / kern_avg_s / 5.0e10,
                         "kernel_ms_mean": kern_avg_s * 1e3,
                         "kernel_ms_min": min(kern_ms)},
            "build_s": build_s,
            "replicate": args.replicate if world > 1 else "single",
            "replicate_s": replicate_s,
            "found_frac": found / B,
        }

    # ---- locate (fm_index.cpp:107-157) on a prefix of the batch, N=1 only ----
    if rank == 0 and world == 1 and args.locate_batch:
        Lq = min(args.locate_batch, B)
        d_sp = torch.empty(Lq, dtype=torch.int64, device=dev)
        d_oo = torch.empty(Lq + 1, dtype=torch.int64, device=dev)
        lt = []
        for it in range(3):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            tot = idx.locate_ranges_device(pats.data_ptr(), offs.data_ptr(), Lq, 100000,
                                           d_sp.data_ptr(), d_oo.data_ptr(), sh)
            if it == 0:
                d_pos = torch.empty(max(tot, 1), dtype=torch.int64, device=dev)
            idx.locate_walk_device(d_sp.data_ptr(), d_oo.data_ptr(), Lq, tot, d_pos.data_ptr(), sh)
            torch.cuda.synchronize()
            lt.append(time.perf_counter() - t1)
        tl = min(lt)
        # every reported position spells its pattern (full-size property check)
        pos = d_pos[:tot]
        oo = d_oo.cpu().numpy()
        owner = torch.from_numpy(np.repeat(np.arange(Lq), np.diff(oo).astype(np.int64))).to(dev)
        win = text[(pos.unsqueeze(1) + torch.arange(m, device=dev)).long()]
        ok = bool((win == pats.view(B, m)[owner]).all().item())
        res["locate"] = {"patterns": Lq, "positions": int(tot), "seconds": tl,
                         "patterns_per_s": Lq / tl, "positions_per_s": tot / tl,
                         "limit": 100000, "positions_verified": ok}
        del d_sp, d_oo, d_pos, owner, win

    # ---- the same batch as one-length k-mers back to back (cs_fm_count_fixed_device: no
    #      offsets array to read), N=1 only: reported beside value, never as value ----
    if rank == 0 and world == 1:
        fo = torch.empty(B, dtype=torch.int64, device=dev)
        for k in range(max(args.warmup, 1)):
            idx.count_fixed_device(pats.data_ptr(), m, B, fo.data_ptr(), sh)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for k in range(args.steps):
            idx.count_fixed_device(pats.data_ptr(), m, B, fo.data_ptr(), sh)
        torch.cuda.synchronize()
        tf = (time.perf_counter() - t1) / args.steps
        res["count_fixed"] = {"patterns": B, "m": m, "ms_per_step": tf * 1e3,
                              "patterns_per_s": B / tf,
                              "matches_batch": bool(np.array_equal(fo.cpu().numpy(), counts))}
        del fo

    # ---- the same batch handed over in host memory (cs_fm_count_batch: PCIe in and out
    #      inside the call), N=1 only: reported beside value, never as value ----
    if rank == 0 and world == 1 and args.host_batch:
        hbuf = pats.cpu().numpy()
        hoffs = offs.cpu().numpy().astype(np.uint64)
        ht = []
        for it in range(3):
            t1 = time.perf_counter()
            hc = idx.count_batch(buf=hbuf, offs=hoffs)
            ht.append(time.perf_counter() - t1)
        res["host_batch"] = {"patterns": B, "seconds": min(ht), "patterns_per_s": B / min(ht),
                             "h2d_bytes": int(hbuf.nbytes + hoffs.nbytes),
                             "matches_device_batch": bool(np.array_equal(hc, counts.astype(np.uint64)))}
        del hbuf, hoffs, hc

    # ---- extract (fm_index.cpp:163-167) on the device, N=1 ----
    if rank == 0 and world == 1 and args.extract_batch:
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
        res["extract"] = {"queries": K_, "len": XL, "seconds": min(xt),
                          "queries_per_s": K_ / min(xt), "bytes_per_s": K_ * XL / min(xt),
                          "verified": bool(torch.equal(want, xout)),
                          "method": ("copy from the text in HBM (text_.substr)" if info.text_in_hbm
                                     else "LF inversion from inverse-SA samples")}
        del xpos, xlen, xoff, xout, want

    # ---- p50 single-pattern latency (>= 1000 single-pattern calls
    #      through the C++ facade, end to end, as tools/benchmark.cpp:154-166) ----
    if rank == 0 and args.p50_calls:
        import ctypes as C
        hp = np.ascontiguousarray(pats[: args.p50_calls * m].cpu().numpy())
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
        res["p50_method"] = ("cs::FMIndex::count via the C++ facade in serving mode "
                             "(FMIndex::serve), %d calls, steady_clock" % nq)
        res["p50_launch_us"] = float(np.median(lat_launch))
        res["p95_launch_us"] = float(np.percentile(lat_launch, 95))
        # the same through the Python mirror (ctypes), for reference
        lat_py = []
        for q in range(min(nq, 1000)):
            b = hp[q * m:(q + 1) * m].tobytes()
            t1 = time.perf_counter()
            idx.count(b)
            lat_py.append((time.perf_counter() - t1) * 1e6)
        res["p50_python_us"] = float(np.median(lat_py))
        res["in_batch_us_per_query"] = elapsed / args.steps / B * 1e6

    # ---- CPU baseline: reference-faithful restatement on host cores (rank 0, N=1) ----
    if args.cpu_queries is None:
        args.cpu_queries = 256 if N <= 200_000_000 else 32 if N <= 2_000_000_000 else 16
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_queries > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline / checker only
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        t1 = time.perf_counter()
        d_bwt = torch.empty(N, dtype=torch.uint8, device=dev)
        idx.bwt_device(d_bwt.data_ptr(), sh)
        bwt = d_bwt.cpu().numpy()
        del d_bwt
        ref = O.Index(bwt=bwt, nthreads=threads)
        del bwt
        prep_s = time.perf_counter() - t1
        Q = args.cpu_queries
        sample = pats[: Q * m].cpu().numpy()
        soffs = np.arange(0, (Q + 1) * m, m, dtype=np.uint64)
        nt = min(threads, Q)
        t1 = time.perf_counter()
        cnt, lat = ref.count_batch(buf=sample, offs=soffs, nthreads=nt, faithful=True,
                                   latencies=True)
        cpu_s = time.perf_counter() - t1
        port = {
            "value": Q / cpu_s, "unit": "patterns/s", "cores": nt, "kind": "port",
            "sample": "first %d patterns of the batch, reference-faithful count() "
                      "(oracle/fm_oracle.c faithful=1), %d host threads" % (Q, nt),
            "p50_us": float(np.median(lat) / 1e3), "seconds": cpu_s, "prep_s": prep_s,
            "matches_gpu": bool(np.array_equal(cnt, counts[:Q].astype(np.uint64)))}
        res["cpu_baseline"] = port
        # the genuine reference's FMIndex::count (oracle/_ref/libcs_ref.so, built from
        # the reference's sources) over its own BitVector tables of the same BWT
        if O.ref_lib() is not None:
            t1 = time.perf_counter()
            gref = O.RefCountIndex(ref)
            rprep = time.perf_counter() - t1
            t1 = time.perf_counter()
            rcnt, rlat = gref.count_batch(sample, soffs, nthreads=nt, latencies=True)
            ref_s = time.perf_counter() - t1
            del gref
            res["cpu_baseline"] = {
                "value": Q / ref_s, "unit": "patterns/s", "cores": nt, "kind": "reference",
                "sample": "first %d patterns of the batch, the reference's own FMIndex::count "
                          "(src/api/fm_index.cpp:79-101, oracle/_ref/libcs_ref.so) over its "
                          "BitVector tables of the same BWT, %d host threads" % (Q, nt),
                "p50_us": float(np.median(rlat) / 1e3), "seconds": ref_s,
                "prep_s": prep_s + rprep,
                "matches_gpu": bool(np.array_equal(rcnt, counts[:Q].astype(np.uint64)))}
            res["cpu_port"] = port
        # also the restatement's fast multi-threaded path (precomputed
        # count_ones totals, the same wavelet rank) over a larger slice of the batch
        Qf = min(args.cpu_fast_queries, B)
        if Qf > 0:
            fs = pats[: Qf * m].cpu().numpy()
            foffs = np.arange(0, (Qf + 1) * m, m, dtype=np.uint64)
            t1 = time.perf_counter()
            fcnt = ref.count_batch(buf=fs, offs=foffs, nthreads=threads, faithful=False)
            fast_s = time.perf_counter() - t1
            res["cpu_fast"] = {
                "value": Qf / fast_s, "unit": "patterns/s", "cores": threads, "kind": "port",
                "sample": "first %d patterns of the batch, oracle count() with precomputed "
                          "totals (not the reference's cost model), %d host threads" % (Qf, threads),
                "seconds": fast_s, "matches_gpu": bool(np.array_equal(fcnt, counts[:Qf].astype(np.uint64)))}
        del ref

    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
