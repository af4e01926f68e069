#!/bin/bash
# round-4 GPU step ao: the driver's bench command with the clock-settle phase
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04ao_bench.json 2> gpurun_out/r04ao_bench.err || exit $?
