#!/bin/bash
# round-4 GPU step i: C4 CG kernel trace (gaps), tiled vs untiled pattern SpMV A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04i_c4_trace -o run -- python3 tools/c4_probe.py 463 50 > gpurun_out/r04i_c4_trace.log 2>&1 || exit $?
AFEM_SPMV_TILE=0 timeout -k 10 200 python3 -u tools/c4_probe.py 463 50 > gpurun_out/r04i_c4_notile.json 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/c4_probe.py 463 50 > gpurun_out/r04i_c4_tile.json 2>&1 || exit $?
