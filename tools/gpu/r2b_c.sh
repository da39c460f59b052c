# split-row BSR kernel: XCD part interleave x non-temporal value staging
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r2b_c
CW=1,2 JB=3 NT=256 ILV=1,2,4 NTV=0,1 NCOLS=8,12,16,24 timeout -k 10 200 python3 $R/tools/bsr_split_sweep.py > $R/gpurun_out/r2b_c/sweep.txt 2>&1
echo done
