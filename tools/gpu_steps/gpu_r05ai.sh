#!/bin/bash
# round-5 GPU step ai: the module's element compiled with -freciprocal-math (the 12 gradient divisions by one
# volume become one reciprocal and multiplies) -- an A/B of the build flag, not the default
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/generic_ab.py 215 10 - - > gpurun_out/r05ai_default.log 2>&1 || exit $?
AFEM_GENERIC_LIB=$PWD/examples/libafem_generic_example_rcp.so timeout -k 10 400 python3 -u tools/generic_ab.py 215 10 - - > gpurun_out/r05ai_rcp.log 2>&1 || exit $?
