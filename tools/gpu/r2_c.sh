cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 120 ./tools/capi_overhead > gpurun_out/r2_capi2.log 2>&1 &&
timeout -k 10 120 ./tools/capi_overhead permute 16 64 5 >> gpurun_out/r2_capi2.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_copy.py tests/test_gpu_golden.py tests/test_gpu_scale.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2_copy_tests.log 2>&1 &&
timeout -k 10 300 python tools/bsr_order.py > gpurun_out/r2_bsr_order.log 2>&1
