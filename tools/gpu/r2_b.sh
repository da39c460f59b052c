cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 120 ./tools/capi_overhead > gpurun_out/r2_capi.log 2>&1 &&
timeout -k 10 120 ./tools/capi_overhead permute 16 64 5 >> gpurun_out/r2_capi.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_golden.py tests/test_gpu_copy.py -m gpu -q --timeout 450 --timeout-method thread > gpurun_out/r2_dist_tests.log 2>&1 ;
echo "pytest rc=$?" >> gpurun_out/r2_dist_tests.log
