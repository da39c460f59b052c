# round 6 aa: tall-skinny updates n = k = 32 / 64 on the fragment kernel (gemm.frag_tall) against
# the tiled kernels, complex<double> and complex<float>
set -o pipefail
O=gpurun_out/r06aa
mkdir -p $O
for dt in cfloat cdouble; do
DTYPE=$dt KINDS=update SIZES=24,32,48,64 FRAGS=1 TALLS=16,32,64 timeout -k 10 300 python3 -u tools/studies/gemm_skinny_bench.py >> $O/tall.txt 2>&1 || { tail -20 $O/tall.txt; exit 1; }
done
grep -v amdgpu.ids $O/tall.txt
