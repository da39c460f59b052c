# round 3: full GPU suite (runtime flags, cache cap, N=2 bench self-check) on the new tree
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_b &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3_b/gpu_tests.log 2>&1
