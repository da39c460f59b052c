set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dense_io.py tests/test_gpu_gemm.py -k "many_rhs or skinny or host_context or trsm" > gpurun_out/r06a/tests.txt 2>&1 || { echo TESTS_FAILED; exit 1; }
tail -2 gpurun_out/r06a/tests.txt
export OMP_NUM_THREADS=16
( time timeout -k 10 1000 tests/refcallers/bin/contract ) > gpurun_out/r06a/contract_full.txt 2>&1
echo "rc=$?" >> gpurun_out/r06a/contract_full.txt
tail -5 gpurun_out/r06a/contract_full.txt
