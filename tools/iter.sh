#!/bin/bash
# Quick GPU iteration on the assembly kernel: parity tests, bench line, and
# one PMC pass of LDS / wait counters (each step under its own time limit).
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --steps 20 --warmup 3 --cg-iters 2 --no-cpu-baseline --no-extras"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
timeout -k 10 200 python3 $B > gpurun_out/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); r=d['roofline']; print('value', d['value'], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'])"
K=${K:-k_assemble}
timeout -k 5 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "$K" -f csv -d gpurun_out/pmc1 -o run -- python3 bench.py --steps 4 --warmup 1 --cg-iters 2 --no-cpu-baseline --no-extras > gpurun_out/pmc1.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc1 | grep mean
timeout -k 5 150 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/trace -o run -- python3 bench.py --steps 6 --warmup 1 --cg-iters 2 --no-cpu-baseline --no-extras > gpurun_out/trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
python3 - <<'PY'
import csv
for x in csv.DictReader(open('gpurun_out/trace/run_kernel_stats.csv')):
    if 'assemble' in x['Name'] or 'strip' in x['Name']: print(x['Name'][:90], x['Calls'], x['AverageNs'])
rows=[x for x in csv.DictReader(open('gpurun_out/trace/run_kernel_trace.csv')) if 'assemble' in x['Kernel_Name']]
x=rows[-1]; print({k:x[k] for k in ['VGPR_Count','Accum_VGPR_Count','SGPR_Count','Grid_Size_X']})
PY
