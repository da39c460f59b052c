# round 6 ae: 128 x 64 LDS-DMA tiles (gemm.tall64) for 33-64 output columns: updates and inner
# products n = 48 / 64, complex<float> and complex<double>, against the 64 x 64 tiles
set -o pipefail
O=gpurun_out/r06ae
mkdir -p $O
for dt in cfloat cdouble; do
DTYPE=$dt KINDS=update,inner SIZES=48,64 FRAGS=1 TALL64=0,1,0,1 timeout -k 10 300 python3 -u tools/studies/gemm_skinny_bench.py >> $O/t64.txt 2>&1 || { tail -20 $O/t64.txt; exit 1; }
done
grep -v amdgpu.ids $O/t64.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['dtype'], d['kind'], d['m'], d['n'], d['k'], 'tall64', d['tall64'], d['us'], d['TBps'])"
