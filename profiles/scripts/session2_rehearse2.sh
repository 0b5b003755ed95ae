# session 2: 2-rank rehearsal of the multi-GPU bench path on one GPU (gloo), on a C2-size
# text: two C4 builds at once do not fit one GPU (each rank's build peaks at ~100 GB);
# on a node every rank has its own GPU.  Then the broadcast replication path at C2 size.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --no-cpu --steps 20 --text-bytes 99999999 --batch 1000000 > gpurun_out/s2_rehearse2.json 2> gpurun_out/s2_rehearse2.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --dist-backend gloo --no-cpu --steps 20 --text-bytes 99999999 --batch 1000000 --replicate broadcast --gather > gpurun_out/s2_rehearse2_bcast.json 2> gpurun_out/s2_rehearse2_bcast.err
