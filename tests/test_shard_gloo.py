"""Multi-process (world_size 2 and 3, gloo, CPU) test of the query-sharding path
used by bench.py on N GPUs: contiguous shards, local count, gather to rank 0, and
the variable-length gather for located positions.  The per-shard engine here is
the oracle stand-in (the HIP engine needs a GPU); the collective plumbing is the
same code (shard.py)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, result_path):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import load_pkg
    import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import importlib
    load_pkg()
    shard = importlib.import_module("cs_fmindex_amd.shard")
    text = O.gen_dna(5, 50_000)
    idx = O.Index(text.tobytes())  # replicated index (stand-in engine)
    pats = O.gen_patterns_text(text, 20, total, seed=4242)

    def count_fn(lo, hi):
        buf = np.ascontiguousarray(pats[lo:hi]).reshape(-1)
        offs = np.arange(0, (hi - lo + 1) * 20, 20, dtype=np.uint64)
        return torch.from_numpy(idx.count_batch(buf=buf, offs=offs).astype(np.int64))

    full = shard.sharded_count(count_fn, total, world, rank, torch.device("cpu"))
    lo, hi = shard.shard_range(total, rank, world)
    # variable-length gather of located positions of the shard's first patterns
    pos = []
    for q in range(lo, min(hi, lo + 5)):
        pos += idx.locate(pats[q].tobytes())
    parts = shard.gather_v(torch.tensor(pos, dtype=torch.int64), world, rank)
    # pipelined, double-buffered gather over 5 steps of equal shards (bench.py N > 1)
    per = (total + world - 1) // world
    pg = shard.PipelinedGather(per, world, rank, torch.int64, torch.device("cpu"))
    for k in range(5):
        buf = pg.buffer(k)
        buf.zero_()
        v = count_fn(lo, hi) + k
        buf[: v.numel()] = v
        pg.submit(k)
        if k == 2:
            pg.finish()
            step2 = pg.result(2)
            step2 = None if step2 is None else step2.clone()
    pg.finish()
    last = pg.result(4)
    # the counts' wire form (cs_counts_pack_wire's layout, packed here by the test since the
    # packer is a HIP kernel) through the pipelined gather, decoded by shard.unpack_counts;
    # counts >= 255 travel as pairs
    cap = 4
    nbw = 16 + 16 * cap + ((per + 7) // 8) * 8
    pw = shard.PipelinedGather(nbw, world, rank, torch.uint8, torch.device("cpu"))
    wire_ok = True
    for k in range(3):
        v = np.zeros(per, np.int64)
        v[: hi - lo] = count_fn(lo, hi).numpy() * (1 + 200 * k) + rank
        w = pw.buffer(k)
        w.zero_()
        big = np.nonzero(v >= 255)[0][:cap]
        hdr = np.array([len(np.nonzero(v >= 255)[0]), cap], np.uint64)
        w[:16] = torch.from_numpy(hdr.view(np.uint8))
        pr = np.stack([big, v[big]], axis=1).astype(np.uint64).reshape(-1)
        w[16:16 + 16 * len(big)] = torch.from_numpy(pr.view(np.uint8))
        w[16 + 16 * cap:16 + 16 * cap + per] = torch.from_numpy(np.minimum(v, 255).astype(np.uint8))
        pw.submit(k)
        pw.finish()
        parts_w = pw.result_parts(k)
        if rank == 0:
            for r in range(world):
                a, b = shard.shard_range(total, r, world)
                want_r = np.zeros(per, np.int64)
                want_r[: b - a] = np.array([idx.count(bytes(pats[q])) for q in range(a, b)],
                                           np.int64) * (1 + 200 * k) + r
                try:
                    got_r = shard.unpack_counts(parts_w[r], per).numpy()
                    wire_ok &= bool(np.array_equal(got_r, want_r))
                except OverflowError:
                    wire_ok &= int((want_r >= 255).sum()) > cap
    if rank == 0:
        want = idx.count_batch([bytes(p) for p in pats]).astype(np.int64)
        ok = bool(np.array_equal(full.numpy(), want))
        for k, got in ((2, step2), (4, last)):
            parts_k = [got[r * per:(r + 1) * per][: max(0, shard.shard_range(total, r, world)[1]
                                                         - shard.shard_range(total, r, world)[0])]
                       for r in range(world)]
            ok &= bool(np.array_equal(torch.cat(parts_k).numpy(), want + k))
        want_pos = []
        for r in range(world):
            a, b = shard.shard_range(total, r, world)
            v = []
            for q in range(a, min(b, a + 5)):
                v += idx.locate(pats[q].tobytes())
            want_pos.append(v)
        ok &= [p.tolist() for p in parts] == want_pos
        ok &= wire_ok
        with open(result_path, "w") as f:
            f.write("ok" if ok else "mismatch")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 1000), (3, 1001), (2, 1)])
def test_sharded_count_gloo(tmp_path, world, total):
    res = tmp_path / "res.txt"
    mp.start_processes(_worker, args=(world, _free_port(), total, str(res)), nprocs=world,
                       join=True, start_method="spawn")
    assert res.read_text() == "ok"


def test_shard_range_partition():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import load_pkg
    import importlib
    load_pkg()
    shard = importlib.import_module("cs_fmindex_amd.shard")
    for total in (0, 1, 7, 100, 101):
        for world in (1, 2, 3, 8):
            rs = [shard.shard_range(total, r, world) for r in range(world)]
            cover = [i for a, b in rs for i in range(a, b)]
            assert cover == list(range(total))
