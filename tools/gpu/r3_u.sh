# round 3: the site-block transpose with paired 16-byte accesses for 8-byte elements
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_u && O=gpurun_out/r3_u &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_copy_trans.py tests/test_gpu_copy.py tests/test_gpu_golden.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
PERMUTE_CONFIGS='[{}, {"trans": -1}]' timeout -k 10 200 python tools/permute_sweep.py > $O/permute_sweep.txt 2>&1
