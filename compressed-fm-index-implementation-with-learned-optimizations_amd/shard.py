"""Multi-GPU query sharding.

One process per GPU, the index replicated in every GPU's HBM, the query batch
split into contiguous ranges, per-shard results gathered to rank 0 over the
process group (RCCL over xGMI on the GPU box; gloo in the CPU tests).  No text
sharding: a query never needs another GPU's data, so the only collective is the
final gather.

The helpers are engine-agnostic: `count_fn(lo, hi) -> tensor[hi-lo]` runs the
local shard (the HIP engine in bench.py; the oracle stand-in in the gloo tests).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous range of ceil(total/world) queries for `rank` (the last shards may
    be shorter or empty)."""
    per = (total + world - 1) // world
    lo = min(total, rank * per)
    hi = min(total, lo + per)
    return lo, hi


def gather_counts(local: torch.Tensor, total: int, world: int, rank: int, dst: int = 0):
    """Gather every rank's shard of a length-`total` result vector to `dst`.

    Shards follow shard_range; each is padded to the common shard length so the
    collective is a plain gather.  Returns the full vector on dst, else None."""
    per = (total + world - 1) // world
    buf = torch.zeros(per, dtype=local.dtype, device=local.device)
    buf[: local.numel()] = local
    if world == 1:
        return buf[:total]
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, parts, dst=dst)
    if rank != dst:
        return None
    return torch.cat(parts)[:total]


def gather_v(local: torch.Tensor, world: int, rank: int, dst: int = 0):
    """Gather variable-length 1-D tensors (e.g. located positions) to dst: an
    all_gather of the lengths, then a padded gather.  Returns the list of per-rank
    tensors on dst, else None."""
    if world == 1:
        return [local]
    n = torch.tensor([local.numel()], dtype=torch.int64,
                     device="cpu" if dist.get_backend() == "gloo" else local.device)
    lens = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(lens, n)
    lens = [int(x.item()) for x in lens]
    mx = max(lens) if lens else 0
    # gloo gathers host tensors only (the N-rank rehearsal on one GPU)
    bdev = "cpu" if dist.get_backend() == "gloo" else local.device
    buf = torch.zeros(max(mx, 1), dtype=local.dtype, device=bdev)
    buf[: local.numel()] = local
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, parts, dst=dst)
    if rank != dst:
        return None
    return [p[:l] for p, l in zip(parts, lens)]


class PipelinedGather:
    """Double-buffered gather of fixed-size shards, overlapped with compute.

    Step k writes its shard into buffer(k) (which first waits for the gather that
    last used that buffer) and submit(k) starts an asynchronous gather of it to dst.
    On the GPU the count kernel of step k+1 (compute stream) runs while the gather
    of step k moves over xGMI (RCCL's stream); finish() waits for every gather.
    """

    def __init__(self, per: int, world: int, rank: int, dtype, device, dst: int = 0, depth: int = 2):
        self.world, self.rank, self.dst, self.depth = world, rank, dst, depth
        self.local = [torch.empty(per, dtype=dtype, device=device) for _ in range(depth)]
        # gloo gathers host tensors only: stage GPU shards through the host (rehearsal
        # of the N-rank path on one GPU; the GPU box's N-GPU runs use RCCL directly)
        self.stage = (world > 1 and torch.device(device).type == "cuda"
                      and dist.get_backend() == "gloo")
        rdev = "cpu" if self.stage else device
        self.recv = ([[torch.empty(per, dtype=dtype, device=rdev) for _ in range(world)]
                      for _ in range(depth)] if rank == dst else [None] * depth)
        self.work = [None] * depth

    def buffer(self, k: int) -> torch.Tensor:
        i = k % self.depth
        if self.work[i] is not None:
            self.work[i].wait()
            self.work[i] = None
        return self.local[i]

    def submit(self, k: int):
        i = k % self.depth
        if self.world == 1:
            return
        src = self.local[i].cpu() if self.stage else self.local[i]
        self.work[i] = dist.gather(src, self.recv[i], dst=self.dst, async_op=True)

    def finish(self):
        for i, w in enumerate(self.work):
            if w is not None:
                w.wait()
                self.work[i] = None

    def result(self, k: int):
        """Gathered vector of step k on dst (valid after finish())."""
        i = k % self.depth
        if self.world == 1:
            return self.local[i]
        return torch.cat(self.recv[i]) if self.rank == self.dst else None

    def result_parts(self, k: int):
        """The per-rank buffers of step k on dst (valid after finish())."""
        i = k % self.depth
        if self.world == 1:
            return [self.local[i]]
        return list(self.recv[i]) if self.rank == self.dst else None


def sharded_count(count_fn, total: int, world: int, rank: int, device, dst: int = 0):
    """Run this rank's contiguous shard with count_fn and gather all to dst."""
    lo, hi = shard_range(total, rank, world)
    local = count_fn(lo, hi) if hi > lo else torch.zeros(0, dtype=torch.int64, device=device)
    return gather_counts(local.to(device), total, world, rank, dst)


def device_bytes(ptr: int, nbytes: int, device) -> torch.Tensor:
    """A uint8 tensor over nbytes of device memory the engine owns (no copy), through
    __cuda_array_interface__: lets a collective send from / receive into the index's
    own parts."""
    class _Arr:
        pass
    a = _Arr()
    a.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                  "strides": None, "version": 2}
    return torch.as_tensor(a, device=device)


def replicate_index(fm, idx, src: int, rank: int, world: int, device):
    """The index built (or opened) on rank `src` on every rank's `device`, at one
    index's worth of HBM per GPU: rank src broadcasts each part of its device image
    straight from the index's own memory (cs_fm_export_part_ptrs), and the other ranks
    receive straight into the parts of a handle allocated for it (cs_fm_import_alloc,
    then cs_fm_import_commit).  RCCL over xGMI with the nccl backend; gloo moves host
    tensors, so there each part is staged through host memory.  `fm` is the package,
    `idx` the FMIndex on src (None on the other ranks).  SURVEY §8(e): replicate by
    broadcast instead of building on every GPU."""
    if world == 1:
        return idx
    stage = dist.get_backend() == "gloo"
    bdev = torch.device("cpu") if stage else torch.device(device)
    if rank == src:
        meta, sizes = idx.export_meta()
        hdr = torch.tensor([len(meta), len(sizes)], dtype=torch.int64, device=bdev)
    else:
        hdr = torch.zeros(2, dtype=torch.int64, device=bdev)
    dist.broadcast(hdr, src)
    meta_len, nparts = int(hdr[0]), int(hdr[1])
    szt = (torch.tensor(sizes, dtype=torch.int64, device=bdev) if rank == src
           else torch.zeros(nparts, dtype=torch.int64, device=bdev))
    dist.broadcast(szt, src)
    sizes = [int(v) for v in szt.tolist()]
    mt = (torch.frombuffer(bytearray(meta), dtype=torch.uint8).to(bdev) if rank == src
          else torch.zeros(meta_len, dtype=torch.uint8, device=bdev))
    dist.broadcast(mt, src)
    meta = bytes(mt.cpu().numpy().tobytes())
    if rank == src:
        out, ptrs = idx, idx.export_part_ptrs(nparts)
    else:
        out, ptrs = fm.FMIndex.import_alloc(meta, nparts, torch.device(device).index)
    for ptr, nb in zip(ptrs, sizes):
        if nb == 0:
            continue
        part = device_bytes(ptr, nb, device)
        if stage:  # gloo moves host tensors only
            h = part.cpu() if rank == src else torch.empty(nb, dtype=torch.uint8)
            dist.broadcast(h, src)
            if rank != src:
                part.copy_(h)
        else:
            dist.broadcast(part, src)
        del part
    torch.cuda.synchronize(device)
    if rank != src:
        out.import_commit()
    return out


# ---- the gathered counts' wire form (cs_counts_pack_wire) -----------------------

WIRE_CAP = 4096  # overflow pairs (counts >= 255) per shard and step


def wire_bytes(fm, per: int, cap: int = WIRE_CAP) -> int:
    return fm.counts_wire_bytes(per, cap)


def pack_counts(fm, counts: torch.Tensor, wire: torch.Tensor, cap: int = WIRE_CAP, stream: int = 0):
    """Pack a device uint64 count vector into `wire` (uint8, wire_bytes long) on the
    GPU: 1 B per count plus the overflow pairs (include/cs_fmindex.h
    cs_counts_pack_wire)."""
    assert counts.is_cuda and wire.is_cuda and counts.dtype == torch.int64
    assert wire.numel() >= fm.counts_wire_bytes(counts.numel(), cap)
    fm.counts_pack_wire(counts.data_ptr(), counts.numel(), cap, wire.data_ptr(), stream)


def unpack_counts(wire: torch.Tensor, npat: int) -> torch.Tensor:
    """The exact int64 counts of one shard's wire form.  Raises when the shard had more
    overflow pairs than its buffer holds (the caller then fetches that shard's counts
    as uint64)."""
    w = wire.reshape(-1)
    hdr = w[:16].view(torch.int64)
    pairs, cap = int(hdr[0].item()), int(hdr[1].item())
    if pairs > cap:
        raise OverflowError("wire: %d counts >= 255, buffer holds %d" % (pairs, cap))
    u8 = w[16 + 16 * cap: 16 + 16 * cap + npat]
    out = u8.to(torch.int64)
    if pairs:
        pr = w[16: 16 + 16 * pairs].view(torch.int64).view(-1, 2)
        out[pr[:, 0]] = pr[:, 1]
    return out
