#!/bin/bash
# round-5 GPU step bb: final state -- the whole suite + smoke, the driver's bench command, then the C2 / C4 /
# unstructured traces + PMC of the final code
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05bb_suite.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05bb_smoke.log 2>&1 || exit $?
timeout -k 10 600 python3 -u bench.py > gpurun_out/r05bb_bench.json 2> gpurun_out/r05bb_bench.err || exit $?
bash tools/profile_legs.sh gpurun_out/r05bb_prof c2 c4 unstructured || exit $?
