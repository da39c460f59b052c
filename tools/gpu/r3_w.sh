# round 3: block transpose kernel -- copy tests, then the named copy shapes with the transpose kernels on / off
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_w && O=gpurun_out/r3_w &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_copy_trans.py tests/test_gpu_copy.py tests/test_gpu_golden.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
COPY_KINDS=1 SBX_COPY_DEBUG=1 timeout -k 10 300 python tools/copy_shapes.py > $O/copy_kinds.txt 2> $O/copy_kinds.err
