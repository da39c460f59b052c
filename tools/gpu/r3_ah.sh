# round 3 (session 2): BSR fuzz across column counts 1-1100 and element types
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_ah && O=gpurun_out/r3_ah &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -k bsr_wide -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
