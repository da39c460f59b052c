# round 3 (session 2): image-side BSR fuzz
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_am && O=gpurun_out/r3_am &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -k image_side -q -rf --timeout 120 --timeout-method thread > $O/tests.log 2>&1
