# split-row BSR kernel: persistent form with prefetched block columns vs the one-chunk form
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r2b_e
CW=1,2 JB=3 NT=256 ILV=2 PK=0,-1,2,3,4,6 NCOLS=8,12,16,24 timeout -k 10 200 python3 $R/tools/bsr_split_sweep.py > $R/gpurun_out/r2b_e/sweep.txt 2>&1
echo done
