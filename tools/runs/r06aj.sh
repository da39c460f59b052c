# round 6 aj: tests/dist.cpp at its default lattice on the final tree (fragment kernel with k pairs,
# NT tiles, tall form to 48 for complex<float>)
set -o pipefail
O=gpurun_out/r06aj
mkdir -p $O
export OMP_NUM_THREADS=16
( time timeout -k 10 500 tests/refcallers/bin/dist ) > $O/dist_default.txt 2>&1
echo "rc=$?" >> $O/dist_default.txt
tail -4 $O/dist_default.txt
