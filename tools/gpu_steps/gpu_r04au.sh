#!/bin/bash
# round-4 GPU step au: final tree -- the whole GPU suite and smoke()
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r04au_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04au_smoke.log 2>&1 || exit $?
