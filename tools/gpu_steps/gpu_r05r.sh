#!/bin/bash
# round-5 GPU step r: host-transport multi-rank rehearsals on one GPU with the per-rank breakdown
# (assembly ms, halo wait and all-reduce ms per CG iteration, halo payload) -- flow checks, not scaling
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u bench.py --gpus 8 --comm host --scaling strong --n 463 --steps 5 --warmup 2 --cg-iters 20 > gpurun_out/r05r_c4_strong8.json 2> gpurun_out/r05r_c4_strong8.err || exit $?
timeout -k 10 400 python3 -u bench.py --gpus 2 --comm host --steps 10 --warmup 3 --cg-iters 20 > gpurun_out/r05r_weak2.json 2> gpurun_out/r05r_weak2.err || exit $?
