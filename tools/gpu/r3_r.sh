# round 3: site-block transpose copy kernel -- its GPU tests, the copy / golden suites, the permute
# sweep with the kernel on and off, the C-ABI eager loop, and the bench line
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_r && O=gpurun_out/r3_r &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_copy_trans.py tests/test_gpu_copy.py tests/test_gpu_golden.py tests/test_gpu_scale.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
PERMUTE_CONFIGS='[{}, {"trans": -1}]' timeout -k 10 200 python tools/permute_sweep.py > $O/permute_sweep.txt 2>&1 &&
timeout -k 10 120 tools/capi_overhead permute 16 64 50 > $O/capi_permute.txt 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err
