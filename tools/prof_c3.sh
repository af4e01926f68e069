# rocprofv3 passes over the C3 leg (run on the GPU box): kernel stats + PMC
set -e
export TMPDIR=/tmp
O=${1:-gpurun_out/c3_prof}
K=${2:-k_assemble_elast}
C="python3 tools/c3_probe.py 170 5"
mkdir -p $O
timeout -k 5 150 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- $C > $O/t.log 2>&1
timeout -k 5 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex $K -f csv -d $O/sq -o run -- $C > $O/s.log 2>&1
timeout -k 5 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $K -f csv -d $O/fetch -o run -- $C > $O/f.log 2>&1
timeout -k 5 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $K -f csv -d $O/write -o run -- $C > $O/w.log 2>&1
timeout -k 5 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-include-regex $K -f csv -d $O/lds -o run -- $C > $O/l.log 2>&1
echo done
