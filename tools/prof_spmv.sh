set -e
export TMPDIR=/tmp
O=gpurun_out/spmv_prof
mkdir -p $O
C="python3 tools/cg_probe.py AFEM_SPMV default --iters 20 --reps 1"
timeout -k 5 120 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- $C > $O/t.log 2>&1
timeout -k 5 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_spmv|k_cg" -f csv -d $O/fetch -o run -- $C > $O/f.log 2>&1
timeout -k 5 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_spmv|k_cg" -f csv -d $O/write -o run -- $C > $O/w.log 2>&1
timeout -k 5 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_spmv" -f csv -d $O/lds -o run -- $C > $O/l.log 2>&1
echo done
