#!/bin/bash
# round-5 GPU step c: where the cube kernel's time goes -- phase ablations (AFEM_CUBES_DIAG) and PC sampling
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab_knobs.py --n 215 --rounds 3 'base:' 'nostore: AFEM_CUBES_DIAG=1' 'oneadd: AFEM_CUBES_DIAG=2' \
  'noarith: AFEM_CUBES_DIAG=4' 'noflush: AFEM_CUBES_DIAG=8' 'nostore+oneadd: AFEM_CUBES_DIAG=3' 'noarith+oneadd: AFEM_CUBES_DIAG=6' \
  'noarith+noflush: AFEM_CUBES_DIAG=12' 'onlyloop: AFEM_CUBES_DIAG=14' 'noflush+nostore: AFEM_CUBES_DIAG=9' > gpurun_out/r05c_diag.log 2>&1 || exit $?
timeout -k 10 60 rocprofv3 -L > gpurun_out/r05c_pcs_list.log 2>&1
timeout -k 10 200 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -f csv -d gpurun_out/r05c_pcs -o run -- python3 bench.py --no-extras --no-cpu-baseline --cg-iters 2 --settle-ms 1000 > gpurun_out/r05c_pcs.log 2>&1
echo "pcs rc=$?" >> gpurun_out/r05c_pcs.log
