#!/bin/bash
# round-4 GPU step av: the multi-rank bench flow with the clock-settle phase (2 ranks, host transport)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u bench.py --gpus 2 --comm host --steps 10 --warmup 3 --cg-iters 20 > gpurun_out/r04av_weak2.json 2> gpurun_out/r04av_weak2.err || exit $?
