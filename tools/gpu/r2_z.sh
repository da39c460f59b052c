cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 450 --timeout-method thread > gpurun_out/r2_gpu_tests4.log 2>&1 &&
NCOLS=1,2,3,4,8,12,16,24,64 timeout -k 10 120 python tools/bsr_probe.py stencil random > gpurun_out/r2_default_probe.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 20 --warmup 10 > gpurun_out/r2_bench4.log 2>&1
