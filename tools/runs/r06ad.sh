# round 6 ad: k pairs with the refined rule: GEMM / golden / contraction tests (pair tests
# included), the complex<float> dist.cpp shapes at the defaults
set -o pipefail
O=gpurun_out/r06ad
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_golden.py tests/test_gpu_contraction.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
DTYPE=cfloat KINDS=inner,update SIZES=8,12,16,32,64 FRAGS=1 timeout -k 10 300 python3 -u tools/studies/gemm_skinny_bench.py > $O/sweep.txt 2>&1 || { tail -20 $O/sweep.txt; exit 1; }
grep -v amdgpu.ids $O/sweep.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['kind'], d['m'], d['n'], d['k'], d['us'], d['TBps'])"
