#!/bin/bash
# Diagnostic: assembly kernel time per ablation mode (results are wrong for modes != 0).
for m in ${MODES:-0 1 2 3 4 5}; do
  AFEM_ASSEMBLY_ABLATION=$m python3 bench.py --steps 20 --warmup 3 --cg-iters 2 --no-cpu-baseline --no-extras | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('mode', $m, 'kernel_ms', d['roofline']['kernel_ms'])"
done
