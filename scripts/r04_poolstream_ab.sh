#!/bin/bash
# C5 schedule: the pool pass on its own stream (event waits both ways) vs in
# order on the pipeline stream
cd "$(dirname "$0")/.."
STEPS=20 bash scripts/ab_env.sh "own||" "pipe||--pool-stream pipe" > gpurun_out/poolstream.txt 2>&1
