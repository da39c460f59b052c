# round 3 (session 2): Kronecker BSR fuzz
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_al && O=gpurun_out/r3_al &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_kron_bsr.py -q -rf --timeout 120 --timeout-method thread > $O/tests.log 2>&1
