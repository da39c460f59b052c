# round 6 ab: the fragment kernel's tall form up to 32 for complex<float>: GEMM / golden /
# contraction GPU tests, and the update sweep at the default
set -o pipefail
O=gpurun_out/r06ab
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_golden.py tests/test_gpu_contraction.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
DTYPE=cfloat KINDS=update,inner SIZES=12,16,24,32,64 FRAGS=1 timeout -k 10 300 python3 -u tools/studies/gemm_skinny_bench.py > $O/sweep.txt 2>&1 || { tail -20 $O/sweep.txt; exit 1; }
grep -v amdgpu.ids $O/sweep.txt | cut -c1-200
