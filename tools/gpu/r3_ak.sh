# round 3 (session 2): the multi-rank tests with the larger distributed fuzz
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_ak && O=gpurun_out/r3_ak &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 450 --timeout-method thread > $O/tests.log 2>&1
