#!/bin/bash
# round-4 GPU step al: final state -- the whole GPU suite, smoke(), the default bench, C2 / C4 profiles
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r04al_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04al_smoke.log 2>&1 || exit $?
timeout -k 10 700 python3 -u bench.py > gpurun_out/r04al_bench.json 2> gpurun_out/r04al_bench.err || exit $?
bash tools/profile_r1.sh gpurun_out/r04al_prof k_assemble_cubes > gpurun_out/r04al_prof.log 2>&1 || exit $?
B="tools/c4_probe.py 463 2 8" bash tools/profile_r1.sh gpurun_out/r04al_prof_c4 k_assemble_cubes > gpurun_out/r04al_prof_c4.log 2>&1 || exit $?
