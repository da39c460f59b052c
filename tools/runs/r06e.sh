# round 6 e: the reference's exhaustive contraction sweep with two components per tensor, and
# tests/dist.cpp at its default lattice (16 16 16 32, n = 64), through the HIP library
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
export OMP_NUM_THREADS=16
( time timeout -k 10 1100 tests/refcallers/bin/contract --components=2 ) > $O/contract_full_c2.txt 2>&1
echo "rc=$?" >> $O/contract_full_c2.txt
tail -6 $O/contract_full_c2.txt
