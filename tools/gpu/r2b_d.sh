# chunk interleave for the row-chunk kernel (n = 32, 64) and the split kernel defaults
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r2b_d
ELL9_ILV=2,4,8 CW=2 JB=3,9 NT=256 ILV=1,2,4 NCOLS=4,12,32,64 timeout -k 10 200 python3 $R/tools/bsr_split_sweep.py > $R/gpurun_out/r2b_d/sweep.txt 2>&1
echo done
