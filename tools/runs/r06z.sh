# round 6 z: on the final tree (gemm_frag_kernel, eventless scratch reuse): the reference's
# exhaustive contraction sweep with one and two components per tensor, and tests/dist.cpp at its
# default lattice, through the HIP library
set -o pipefail
O=gpurun_out/r06z
mkdir -p $O
export OMP_NUM_THREADS=16
( time timeout -k 10 500 tests/refcallers/bin/dist ) > $O/dist_default.txt 2>&1
echo "rc=$?" >> $O/dist_default.txt
tail -4 $O/dist_default.txt
grep -q "rc=0" $O/dist_default.txt || exit 1
( time timeout -k 10 480 tests/refcallers/bin/contract ) > $O/contract_full.txt 2>&1
echo "rc=$?" >> $O/contract_full.txt
tail -6 $O/contract_full.txt
grep -q "rc=0" $O/contract_full.txt || exit 1
( time timeout -k 10 480 tests/refcallers/bin/contract --components=2 ) > $O/contract_full_c2.txt 2>&1
echo "rc=$?" >> $O/contract_full_c2.txt
tail -6 $O/contract_full_c2.txt
