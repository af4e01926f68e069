#!/bin/bash
# round-4 GPU step s: generic unit kernel, XOR-swizzled LDS planes A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_generic.py > gpurun_out/r04s_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/generic_ab.py 215 10 - PAD=-1 - PAD=-1 PAD=1 > gpurun_out/r04s_generic_ab.log 2>&1 || exit $?
