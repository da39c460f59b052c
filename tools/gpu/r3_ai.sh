# round 3 (session 2): copy fuzz over larger permutations (transpose kernels on / off), after the
# site-block transpose tile cap (QT <= 256), and the copy / transpose tests
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_ai && O=gpurun_out/r3_ai &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_copy_trans.py tests/test_gpu_copy.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
