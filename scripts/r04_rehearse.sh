#!/bin/bash
# N > 1 bench path on one GPU (every rank on cuda:0, gloo collectives): the
# digest check, sharding and max-over-ranks timing at this tree
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export VC_BENCH_SHARED_GPU=1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
    > gpurun_out/rehearse.jsonl 2> gpurun_out/rehearse.err
