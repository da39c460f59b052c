# round 6 i: 20-deep GEMM slabs (tests, interleaved A/B on the config-2 GEMM)
set -o pipefail
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py -k "slab20 or loader_forms" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
VARIANTS=8:1,8:1:0:20,0:1:0:20 ROUNDS=6 timeout -k 10 300 python -u tools/studies/gemm_loaders.py > $O/slab20.txt 2>&1 || { tail -20 $O/slab20.txt; exit 1; }
cat $O/slab20.txt
