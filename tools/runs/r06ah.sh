# round 6 ah: the fragment kernel's defaults after the NT / tall-48 rules: GEMM / golden /
# contraction tests, dist.cpp's shapes for both complex types
set -o pipefail
O=gpurun_out/r06ah
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_golden.py tests/test_gpu_contraction.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for dt in cfloat cdouble; do
DTYPE=$dt KINDS=inner,update SIZES=8,12,16,32,48,64 FRAGS=1 timeout -k 10 300 python3 -u tools/studies/gemm_skinny_bench.py >> $O/sweep.txt 2>&1 || { tail -20 $O/sweep.txt; exit 1; }
done
grep -v amdgpu.ids $O/sweep.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['dtype'], d['kind'], d['m'], d['n'], d['k'], d['us'], d['TBps'])"
