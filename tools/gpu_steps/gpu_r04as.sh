#!/bin/bash
# round-4 GPU step as: final state -- whole GPU suite, smoke(), the driver's bench command, kernel traces + PMC
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r04as_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04as_smoke.log 2>&1 || exit $?
timeout -k 10 700 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04as_bench.json 2> gpurun_out/r04as_bench.err || exit $?
B="bench.py --steps 20 --warmup 5 --cg-iters 20 --no-cpu-baseline --no-extras" bash tools/profile_r1.sh gpurun_out/r04as_prof k_assemble_cubes > gpurun_out/r04as_prof.log 2>&1 || exit $?
B="tools/c4_probe.py 463 2 8" bash tools/profile_r1.sh gpurun_out/r04as_prof_c4 k_assemble_cubes > gpurun_out/r04as_prof_c4.log 2>&1 || exit $?
