# round 3 final pass on the current tree: the whole -m gpu suite
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_k &&
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r3_k/gpu_tests.log 2>&1
