#!/bin/bash
# round-5 GPU step ab: the whole GPU suite + smoke on the current tree
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ab_suite.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05ab_smoke.log 2>&1 || exit $?
