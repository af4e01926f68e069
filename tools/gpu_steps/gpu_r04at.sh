#!/bin/bash
# round-4 GPU step at: generic unit kernel with wave-scope ordering: tests + A/B (UN 4 default)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_generic.py tests/test_gpu_shim.py > gpurun_out/r04at_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/generic_ab.py 215 10 - - > gpurun_out/r04at_generic_ab.log 2>&1 || exit $?
