#!/bin/bash
# round-4 GPU step ai: final state -- the whole GPU suite, smoke(), the default bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r04ai_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04ai_smoke.log 2>&1 || exit $?
timeout -k 10 700 python3 -u bench.py > gpurun_out/r04ai_bench.json 2> gpurun_out/r04ai_bench.err || exit $?
