#!/bin/bash
# round-4 GPU step n: cube kernel A/B + generic unit kernel with UN functors in flight
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube or slab" > gpurun_out/r04n_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_generic.py tests/test_gpu_shim.py > gpurun_out/r04n_tests_generic.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/cubes_ab.py 215 20 8 16 32 > gpurun_out/r04n_ab215.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/generic_ab.py 215 10 - UN=1 UN=2 UN=3 UN=4 UN=2,PAD=0 UN=1,PAD=0 AFEM_FUNCTOR_UNITS=8192,UN=3 > gpurun_out/r04n_generic_ab.log 2>&1 || exit $?
PMC_CMD="tools/cubes_ab.py 215 3 16" PMC_PASSES="inst wait" bash tools/profile_pmc.sh gpurun_out/r04n_pmc "k_assemble_cubes"
