#!/bin/bash
# round-5 GPU step n: packed entries with patterns prefetched one group ahead; the unit kernel
# held to 3 waves per SIMD (AFEM_GENERIC_WAVES=3 build) -- A/B in one process per library
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_generic.py -k "packed or oracle" > gpurun_out/r05n_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/generic_ab.py 215 10 - - AFEM_FUNCTOR_PACKED=0 - AFEM_FUNCTOR_PACKED=0 > gpurun_out/r05n_ab.log 2>&1 || exit $?
AFEM_GENERIC_LIB=$PWD/examples/libafem_generic_example_w3.so timeout -k 10 400 python3 -u tools/generic_ab.py 215 10 - - AFEM_FUNCTOR_PACKED=0 - AFEM_FUNCTOR_PACKED=0 > gpurun_out/r05n_ab_w3.log 2>&1 || exit $?
