#!/bin/bash
# round-4 GPU step ag: default bench with the cube kernel, its kernel trace + PMC at C2, and C4 alone
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python3 -u bench.py > gpurun_out/r04ag_bench.json 2> gpurun_out/r04ag_bench.err || exit $?
bash tools/profile_r1.sh gpurun_out/r04ag_prof k_assemble_cubes > gpurun_out/r04ag_prof.log 2>&1 || exit $?
B="tools/c4_probe.py 463 2 8" bash tools/profile_r1.sh gpurun_out/r04ag_prof_c4 k_assemble_cubes > gpurun_out/r04ag_prof_c4.log 2>&1 || exit $?
