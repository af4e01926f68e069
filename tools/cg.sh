#!/bin/bash
# CG/SpMV iteration: linear-system GPU tests, bench CG line per SpMV variant,
# kernel trace of the default variant.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "solve or cg or spmv or linear" > gpurun_out/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
for m in default stream; do
  AFEM_SPMV=$m timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cg-iters 200 --no-cpu-baseline --no-extras > gpurun_out/cg_$m.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/cg_$m.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/cg_$m.log').read().strip().splitlines()[-1]); print('$m', {k:v for k,v in d.items() if k.startswith('cg')})"
done
timeout -k 5 150 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/cgtrace -o run -- python3 bench.py --steps 2 --warmup 1 --cg-iters 50 --no-cpu-baseline --no-extras > gpurun_out/cgtrace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
python3 - <<'PY'
import csv
for x in csv.DictReader(open('gpurun_out/cgtrace/run_kernel_stats.csv')):
    print(x['Name'][:70], x['Calls'], x['AverageNs'], x['Percentage'])
PY
