#!/bin/bash
# round-5 GPU step bq: final state after the non-temporal C3 and unstage stores -- the whole suite + smoke, the
# driver's bench command (its legs now reference the profiles of the same code)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05bq_suite.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05bq_smoke.log 2>&1 || exit $?
timeout -k 10 600 python3 -u bench.py > gpurun_out/r05bq_bench.json 2> gpurun_out/r05bq_bench.err || exit $?
