# round 6 s: 8 waves of 64x32 per 128x128 tile against 16 of 32x32 (tools/studies/gemm_tune ONLY=w8)
set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
ONLY=w8 timeout -k 10 300 tools/studies/gemm_tune 20 > $O/w8.txt 2>&1 || { tail -30 $O/w8.txt; exit 1; }
cat $O/w8.txt
