# round 6 h: gemm_frag_kernel (tests, dist.cpp shape sweep)
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_golden.py tests/test_gpu_contraction.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python -u tools/studies/gemm_skinny_bench.py > $O/skinny.txt 2>&1 || { tail -20 $O/skinny.txt; exit 1; }
cat $O/skinny.txt
