cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_copy.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2_copy_tests.log 2>&1 ;
timeout -k 10 300 python tools/bsr_order.py > gpurun_out/r2_bsr_order.log 2>&1
