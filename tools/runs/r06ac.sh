# round 6 ac: 16-byte k pairs in gemm_frag_kernel (8-byte elements): GEMM tests, then the dist.cpp
# shapes with pairs on / off (complex<float> and complex<double>)
set -o pipefail
O=gpurun_out/r06ac
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_golden.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for pr in 1 0 1 0; do
python3 -c "
import superbblas_amd as sb
" >/dev/null
GEMM_PAIR=$pr DTYPE=cfloat KINDS=inner,update SIZES=8,12,16,32 FRAGS=1 timeout -k 10 300 python3 -u tools/studies/gemm_skinny_bench.py >> $O/sweep_cf_$pr.txt 2>&1 || { tail -20 $O/sweep_cf_$pr.txt; exit 1; }
done
grep -v amdgpu.ids $O/sweep_cf_1.txt | cut -c1-200
echo ---
grep -v amdgpu.ids $O/sweep_cf_0.txt | cut -c1-200
