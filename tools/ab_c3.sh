#!/bin/bash
# A/B of the block-3 (C3) assembly: bench C3 side measurement per environment setting.
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --cg-iters 2 --no-cpu-baseline --c5-steps 1 --c5-n 8 > gpurun_out/ab_c3.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/ab_c3.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_c3.log').read().strip().splitlines()[-1]); c=d['c3']; print(sys.argv[1], 'c3 kernel_ms', c['kernel_ms'], 'frac', c['roofline']['frac'])" "$cfg"
done
