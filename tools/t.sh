export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 0 6 7 8; do
  AFEM_ASSEMBLY_WAVES_PER_CU=$w timeout 100 python3 bench.py --steps 20 --warmup 3 --cg-iters 2 --no-cpu-baseline --no-extras | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('wpc $w', d['roofline']['kernel_ms'])"
done
timeout 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/trace -o run -- python3 bench.py --steps 10 --warmup 2 --cg-iters 2 --no-cpu-baseline --no-extras > gpurun_out/trace.log 2>&1
grep assemble gpurun_out/trace/run_kernel_stats.csv | cut -d, -f2-8
