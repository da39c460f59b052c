# round 6 q: 8 loader waves with the next k-step's fragments read before the current MFMAs (gemm.pf)
set -o pipefail
O=gpurun_out/r06q
mkdir -p $O
VARIANTS="8:1,8:1:0:1" ROUNDS=8 timeout -k 10 300 python3 -u tools/studies/gemm_loaders.py > $O/pf.txt 2>&1 || { tail -30 $O/pf.txt; exit 1; }
cat $O/pf.txt
