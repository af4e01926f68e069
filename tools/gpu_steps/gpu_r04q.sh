#!/bin/bash
# round-4 final state, step q: the default bench (all legs, CPU baselines) and the
# headline's kernel trace + PMC passes (tools/profile_r1.sh)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python3 -u bench.py > gpurun_out/r04q_bench.json 2> gpurun_out/r04q_bench.err || exit $?
bash tools/profile_r1.sh gpurun_out/r04q_prof k_assemble_st > gpurun_out/r04q_prof.log 2>&1
