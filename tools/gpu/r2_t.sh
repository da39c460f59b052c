cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_bsr_tile.py tests/test_gpu_bsr.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_tile_tests.log 2>&1 &&
TILE=1 TILE_MIN=1 timeout -k 10 300 python tools/bsr_probe.py stencil > gpurun_out/r2_tile_probe.log 2>&1 &&
TILE=0 timeout -k 10 300 python tools/bsr_probe.py stencil >> gpurun_out/r2_tile_probe.log 2>&1
