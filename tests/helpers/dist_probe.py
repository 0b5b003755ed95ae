"""A rank process for tests/test_bench_spawn.py: started by bench.spawn_ranks exactly as
bench.py's ranks are (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the environment),
it joins a gloo group, checks the world size and has rank 0 print one JSON line.
PROBE_FAIL_RANK=r makes rank r exit with status 3 before joining (rank 0 then waits in
the rendezvous until spawn_ranks stops it)."""
import json
import os
import sys

import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
if os.environ.get("PROBE_FAIL_RANK") == str(rank):
    sys.exit(3)
print("rank %d stdout chatter" % rank, flush=True)  # only rank 0's stdout reaches stdout
dist.init_process_group("gloo")
assert dist.get_world_size() == world == int(sys.argv[1])
seen = [None] * world
dist.all_gather_object(seen, (rank, int(os.environ["LOCAL_RANK"])))
if rank == 0:
    print(json.dumps({"ranks_seen": dist.get_world_size(), "ranks": seen,
                      "spawned": os.environ.get("CS_BENCH_SPAWNED")}), flush=True)
dist.barrier()
dist.destroy_process_group()
