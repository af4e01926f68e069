#!/bin/bash
# round-5 GPU step bj: kernel trace of the AMG setup + solve on the unstructured system
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r05bj_prof -o run -- \
  python3 -u $GRAFT_REPO_ROOT/tools/amg_probe.py 6 1e-8 - > $GRAFT_REPO_ROOT/gpurun_out/r05bj_amg.log 2>&1 || exit $?
