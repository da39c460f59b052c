cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_contraction.py tests/test_gpu_golden.py tests/test_gpu_scale.py tests/test_gpu_fuzz.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2_gemm_tests.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 20 --warmup 10 > gpurun_out/r2_bench2.log 2>&1 &&
timeout -k 10 400 python tools/bsr_sweep.py > gpurun_out/r2_bsr_sweep.log 2>&1
