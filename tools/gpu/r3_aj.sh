# round 3 (session 2): contraction fuzz at GEMM-kernel sizes
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_aj && O=gpurun_out/r3_aj &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -k contraction_large -q -rf --timeout 120 --timeout-method thread > $O/tests.log 2>&1
