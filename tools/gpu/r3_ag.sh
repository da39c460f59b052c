# round 3 (session 2): BSR tests after the >512-column fallback fix
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_ag && O=gpurun_out/r3_ag &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_bsr.py tests/test_gpu_bsr_split.py tests/test_gpu_lds_tails.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
