# round 3 (session 2): masked copy fuzz
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_an && O=gpurun_out/r3_an &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -k copy_masked -q -rf --timeout 120 --timeout-method thread > $O/tests.log 2>&1
