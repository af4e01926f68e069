#!/bin/bash
# A/B of the CG iteration rate per environment setting (100 fixed iterations on C2).
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cg-iters 200 --no-cpu-baseline --no-extras > gpurun_out/ab_cg.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/ab_cg.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_cg.log').read().strip().splitlines()[-1]); print(sys.argv[1], 'cg iter/s', d['cg_iter_per_s'], 'frac', d['cg_roofline_frac'])" "$cfg"
done
