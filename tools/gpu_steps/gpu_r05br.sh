#!/bin/bash
# round-5 GPU step br: general-slice variants incl. the big-list order
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "general_slice_variants" > gpurun_out/r05br_tests.log 2>&1 || exit $?
