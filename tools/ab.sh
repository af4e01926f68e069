#!/bin/bash
# A/B of assembly variants on the GPU box: parity tests, then bench kernel
# time per environment setting given as arguments ("VAR=val VAR2=val ...").
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --steps 20 --warmup 3 --cg-iters 2 --no-cpu-baseline --no-extras"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
for cfg in "$@"; do
  env $cfg timeout -k 10 100 python3 $B > gpurun_out/ab.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'])" "$cfg"
done
