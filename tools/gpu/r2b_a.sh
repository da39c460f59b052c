# split-row BSR kernel: gather-locality probe and L2 traffic (n = 12), run from the repo root
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r2b_a
NCOLS=8,12,24 timeout -k 10 200 python3 $R/tools/bsr_probe.py stencil self9 random > $R/gpurun_out/r2b_a/probe.txt 2>&1
cd /tmp && export TMPDIR=/tmp
NCOLS=12 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r2b_a/fetch -o run -- python3 $R/tools/bsr_probe.py stencil > /dev/null 2>&1
NCOLS=12 timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/r2b_a/hit -o run -- python3 $R/tools/bsr_probe.py stencil > /dev/null 2>&1
NCOLS=12 timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r2b_a/ta -o run -- python3 $R/tools/bsr_probe.py stencil > /dev/null 2>&1
NCOLS=12 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/r2b_a/sq -o run -- python3 $R/tools/bsr_probe.py stencil > /dev/null 2>&1
echo done
