#!/bin/bash
# PC sampling of the assembly (host-trap, time based) on the GPU box.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/pcs_list.log 2>&1
M=${1:-host_trap}
timeout -k 10 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit ${2:-time} --pc-sampling-interval ${3:-1} -f csv -d gpurun_out/pcs -o run -- python3 bench.py --steps 20 --warmup 2 --cg-iters 2 --no-cpu-baseline --no-extras > gpurun_out/pcs.log 2>&1
echo "rc=$?"
ls -la gpurun_out/pcs/ 2>/dev/null | head; find gpurun_out/pcs -type f | head
