#!/bin/bash
# round-4 GPU step o: generic unit kernel UN sweep with dense planes; cube kernel (reverted) A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_generic.py tests/test_gpu_shim.py > gpurun_out/r04o_tests_generic.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/generic_ab.py 215 10 - UN=2 UN=3 UN=4 UN=6 UN=8 UN=4,PAD=1 AFEM_FUNCTOR_UNITS=32768,UN=4 AFEM_FUNCTOR_UNITS=8192,UN=4 > gpurun_out/r04o_generic_ab.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/cubes_ab.py 215 20 8 16 > gpurun_out/r04o_ab215.log 2>&1 || exit $?
