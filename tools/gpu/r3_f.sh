# round 3: full GPU suite after the prune
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_f &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3_f/gpu_tests.log 2>&1
