# round 6 ag: gemm_frag_kernel with NT tiles per wave along n: tests, then updates n = k = 24-64 and
# inner products 32 / 64 with NT 1 / 2 / 4 (tall form to 64), both complex types
set -o pipefail
O=gpurun_out/r06ag
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py -k "frag" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for dt in cfloat cdouble; do
DTYPE=$dt KINDS=update SIZES=24,32,48,64 FRAGS=1 TALLS=64 NTS=1,2,4 timeout -k 10 300 python3 -u tools/studies/gemm_skinny_bench.py >> $O/nt.txt 2>&1 || { tail -20 $O/nt.txt; exit 1; }
DTYPE=$dt KINDS=inner SIZES=32 FRAGS=1 NTS=1,2 timeout -k 10 300 python3 -u tools/studies/gemm_skinny_bench.py >> $O/nt.txt 2>&1 || { tail -20 $O/nt.txt; exit 1; }
done
grep -v amdgpu.ids $O/nt.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['dtype'], d['kind'], d['m'], d['n'], d['k'], 'nt', d['frag_nt'], 'tall', d['frag_tall'], d['us'], d['TBps'])"
