cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 450 --timeout-method thread > gpurun_out/r2_gpu_tests3.log 2>&1 ;
echo "pytest rc=$?" >> gpurun_out/r2_gpu_tests3.log ;
timeout -k 10 400 python bench.py --steps 20 --warmup 10 > gpurun_out/r2_bench3.log 2>&1
