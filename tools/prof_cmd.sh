# rocprofv3 passes over any command (run on the GPU box): kernel stats, then
# separate --pmc passes (SQ timing, FETCH_SIZE, WRITE_SIZE, LDS) restricted to
# the kernels matching $2.  usage: bash tools/prof_cmd.sh OUT KERNEL_REGEX cmd args...
set -e
export TMPDIR=/tmp
O=$1; K=$2; shift 2
mkdir -p $O
timeout -k 5 200 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- "$@" > $O/t.log 2>&1
timeout -k 5 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex $K -f csv -d $O/sq -o run -- "$@" > $O/s.log 2>&1
timeout -k 5 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $K -f csv -d $O/fetch -o run -- "$@" > $O/f.log 2>&1
timeout -k 5 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $K -f csv -d $O/write -o run -- "$@" > $O/w.log 2>&1
timeout -k 5 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-include-regex $K -f csv -d $O/lds -o run -- "$@" > $O/l.log 2>&1
echo done
