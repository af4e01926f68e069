#!/bin/bash
# round-5 GPU step l: packed plan entries of the generic unit kernel (8 B {cell, pattern}), the
# canonical cube flush's 16-B row stores by default; A/B of packing, the XOR swizzle and UN
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_generic.py tests/test_gpu_shim.py > gpurun_out/r05l_tests_generic.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube or canonical or natural or random" > gpurun_out/r05l_tests_cubes.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/generic_ab.py 215 10 - AFEM_FUNCTOR_PACKED=0 PAD=-1 UN=6 UN=3 AFEM_FUNCTOR_PACKED=0,PAD=-1 > gpurun_out/r05l_generic_ab.log 2>&1 || exit $?
