#!/bin/bash
# round-5 GPU step ac: the default bench line, then rocprof evidence (kernel trace with a 1.5-s settle,
# FETCH_SIZE, WRITE_SIZE passes) for the headline C2, C4 and C3 legs
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u bench.py > gpurun_out/r05ac_bench.json 2> gpurun_out/r05ac_bench.err || exit $?
bash tools/profile_legs.sh gpurun_out/r05ac_prof c2 c4 c3 || exit $?
