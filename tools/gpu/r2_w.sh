cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_bsr_tile.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_tile_tests.log 2>&1 &&
NCOLS=12,64 timeout -k 10 300 python tools/bsr_timeline.py > gpurun_out/r2_timeline.log 2>&1
