#!/bin/bash
# round-5 GPU step j: the whole suite + smoke, the driver's bench command, then every leg's trace + PMC
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05j_tests.log 2>&1
RC=$?
[ $RC -ge 124 ] && exit $RC
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05j_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05j_bench.json 2> gpurun_out/r05j_bench.err || exit $?
bash tools/profile_legs.sh gpurun_out/r05j_prof c2 c4 c2_arrays_natural c3 c2_generic c2_arrays unstructured generic_unstructured || exit $?
PASSES="sq lds" bash tools/profile_legs.sh gpurun_out/r05j_prof c2 c3 || exit $?
exit $RC
