#!/bin/bash
# round-5 GPU step a: the whole GPU suite (new: natural-numbering cube path, mapped-view checks,
# duplicate diagonals, slab z segments), the default bench, then C2 / C4 / natural traces + PMC.
# Test failures do not stop the bench (only a time limit, an abort or a crash does).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05a_tests.log 2>&1
RC=$?
[ $RC -ge 124 ] && exit $RC
timeout -k 10 400 python3 -u bench.py > gpurun_out/r05a_bench.json 2> gpurun_out/r05a_bench.err || exit $?
bash tools/profile_legs.sh gpurun_out/r05a_prof c2 c2_arrays_natural c4 || exit $?
exit $RC
