# round 6 ai: inner products m = n = 48 / 64 on the fragment kernel (gemm.frag_small 64, NT 1 / 2 / 4)
# against the tiled kernels, both complex types
set -o pipefail
O=gpurun_out/r06ai
mkdir -p $O
for dt in cfloat cdouble; do
DTYPE=$dt KINDS=inner SIZES=48,64 FRAGS=1 SMALL=32 NTS=0 timeout -k 10 300 python3 -u tools/studies/gemm_skinny_bench.py >> $O/small.txt 2>&1 || { tail -20 $O/small.txt; exit 1; }
DTYPE=$dt KINDS=inner SIZES=48,64 FRAGS=1 SMALL=64 NTS=1,2,4 timeout -k 10 300 python3 -u tools/studies/gemm_skinny_bench.py >> $O/small.txt 2>&1 || { tail -20 $O/small.txt; exit 1; }
done
grep -v amdgpu.ids $O/small.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['dtype'], d['kind'], d['m'], d['n'], d['k'], 'nt', d['frag_nt'], d['us'], d['TBps'], d['TFLOPs'])"
