# round 6 f: tests/dist.cpp at its default lattice (16 16 16 32, n = 64) through the HIP library
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
export OMP_NUM_THREADS=16
( time timeout -k 10 900 tests/refcallers/bin/dist ) > $O/dist_default.txt 2>&1
echo "rc=$?" >> $O/dist_default.txt
tail -40 $O/dist_default.txt
