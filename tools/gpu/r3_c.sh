# round 3: new tests (LDS tails, runtime flags, skipped blocks, N=2 bench self-check)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_c &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_lds_tails.py tests/test_gpu_bsr.py tests/test_gpu_runtime.py tests/test_gpu_dropin.py tests/test_gpu_bench_scale.py -q --timeout 300 --timeout-method thread > gpurun_out/r3_c/tests.log 2>&1
