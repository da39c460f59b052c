set -o pipefail
B=tests/refcallers/bin
export OMP_NUM_THREADS=8
mkdir -p gpurun_out/r5a
timeout -k 10 120 env SB_DEBUG=1 $B/bsr --dim='4 4 4 4 2 3' > gpurun_out/r5a/bsr3.txt 2>&1; echo "bsr3 rc=$?"
timeout -k 10 120 env SB_DEBUG=1 $B/bsr --dim='4 4 4 4 2 12' > gpurun_out/r5a/bsr12.txt 2>&1; echo "bsr12 rc=$?"
for t in 0 1 17 4567 89012 345678 663551 663552 700001 1327103; do timeout -k 10 60 $B/contract --test=$t > gpurun_out/r5a/contract_$t.txt 2>&1; echo "contract $t rc=$?"; done
timeout -k 10 60 $B/contract --test=123457 --components=2 > gpurun_out/r5a/contract_c2.txt 2>&1; echo "contract c2 rc=$?"
timeout -k 10 120 $B/dist --dim='8 8 8 8 8' --reps=2 > gpurun_out/r5a/dist.txt 2>&1; echo "dist rc=$?"
timeout -k 10 120 $B/blas --size=1000 --rep=2 > gpurun_out/r5a/blas.txt 2>&1; echo "blas rc=$?"
timeout -k 10 120 env SB_DEBUG=1 $B/dense --dim='4 4 4 4 2 12' > gpurun_out/r5a/dense.txt 2>&1; echo "dense rc=$?"
grep -h "Caught\|went ok\|rror" gpurun_out/r5a/*.txt | sort | uniq -c
