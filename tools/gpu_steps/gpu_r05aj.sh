#!/bin/bash
# round-5 GPU step aj (final state): the driver's bench command, then C2 (headline command) and C4 traces
# + FETCH_SIZE / WRITE_SIZE passes of the same code
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u bench.py > gpurun_out/r05aj_bench.json 2> gpurun_out/r05aj_bench.err || exit $?
bash tools/profile_legs.sh gpurun_out/r05aj_prof c2 c4 || exit $?
