# round 6 l: gemm_frag_kernel load-group depth and wave count
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
KINDS=inner,update SIZES=8,12,16,32 FRAGS=1 FRAGCFG=4:4096,2:4096,8:4096,4:2048,4:8192,8:8192,4:4096 timeout -k 10 400 python -u tools/studies/gemm_skinny_bench.py > $O/frag_cfg.txt 2>&1 || { tail -20 $O/frag_cfg.txt; exit 1; }
cat $O/frag_cfg.txt
