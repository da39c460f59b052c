# split-row BSR kernel after the division-free index math: sweep + SQ instruction counts (n = 12)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r2b_b
CW=1,2 JB=1,3,9 NT=256,512 NCOLS=4,8,12,16,24,32 timeout -k 10 200 python3 $R/tools/bsr_split_sweep.py > $R/gpurun_out/r2b_b/sweep.txt 2>&1
cd /tmp && export TMPDIR=/tmp
NCOLS=12 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/r2b_b/sq -o run -- python3 $R/tools/bsr_probe.py stencil > /dev/null 2>&1
echo done
