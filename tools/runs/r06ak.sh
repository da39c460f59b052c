# round 6 ak: inner products with an m-contiguous A (dist.cpp's nn / tn forms): B alone paired
# (gemm.frag_pair 2) against unpaired, complex<float>
set -o pipefail
O=gpurun_out/r06ak
mkdir -p $O
for pr in 1 2 1 2; do
GEMM_PAIR=$pr TA_INNER=N DTYPE=cfloat KINDS=inner SIZES=8,12,16,32 FRAGS=1 timeout -k 10 300 python3 -u tools/studies/gemm_skinny_bench.py >> $O/nn_$pr.txt 2>&1 || { tail -20 $O/nn_$pr.txt; exit 1; }
done
for pr in 1 2; do echo "== frag_pair $pr"; grep -v amdgpu.ids $O/nn_$pr.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['kind'], d['m'], d['n'], d['k'], d['us'])"; done
