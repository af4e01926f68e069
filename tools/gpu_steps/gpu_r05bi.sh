#!/bin/bash
# round-5 GPU step bi: AMG after moving the K-cycle kernels to kcycle.hpp (shared with multigrid.hip)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_amg.py tests/test_gpu_multigrid.py \
  > gpurun_out/r05bi_tests.log 2>&1 || exit $?
