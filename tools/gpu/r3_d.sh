# round 3: distributed suite with the collective reduction + N=2 bench self-check
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_d &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_bench_scale.py -v --timeout 450 --timeout-method thread > gpurun_out/r3_d/tests.log 2>&1
