#!/bin/bash
# round-4 GPU step aj: 8-rank host-transport rehearsal of C4 strong scaling with the cube kernel on the slabs,
# and the 2-rank weak rehearsal (two C2 slabs)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u bench.py --gpus 8 --comm host --scaling strong --n 463 --steps 5 --warmup 2 --cg-iters 20 > gpurun_out/r04aj_c4_strong8.json 2> gpurun_out/r04aj_c4_strong8.err || exit $?
timeout -k 10 400 python3 -u bench.py --gpus 2 --comm host --steps 10 --warmup 3 --cg-iters 20 > gpurun_out/r04aj_weak2.json 2> gpurun_out/r04aj_weak2.err || exit $?
