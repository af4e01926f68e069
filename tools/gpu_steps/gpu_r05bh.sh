#!/bin/bash
# round-5 GPU step bh: geometric multigrid with the K-cycle (AFEM_MG_KCYCLE) -- mg tests with it on, C5 A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
AFEM_MG_KCYCLE=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_multigrid.py \
  > gpurun_out/r05bh_tests.log 2>&1 || exit $?
for k in 0 1 2 8; do
  AFEM_MG_KCYCLE=$k timeout -k 10 200 python3 -u tools/c5_probe.py 128 4 > gpurun_out/r05bh_c5_k$k.json 2>&1 || exit $?
done
