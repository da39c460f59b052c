# round 6 j: the dot kernel (m, n <= 4) with 4 k per pass and more workgroups
set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py -k "skinny" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
KINDS=inner SIZES=1,2,4 FRAGS=1 DOTS=256,1024,2048,256,1024,2048 timeout -k 10 300 python -u tools/studies/gemm_skinny_bench.py > $O/dot.txt 2>&1 || { tail -20 $O/dot.txt; exit 1; }
cat $O/dot.txt
