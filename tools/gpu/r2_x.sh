cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_bsr_tile.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_tile_tests.log 2>&1 &&
for r in 16 32 8; do for sl in 32 16 12 8; do NCOLS=4,12,24,64 TROWS=$r SLAB=$sl timeout -k 10 120 python tools/bsr_probe.py stencil || exit 1; done; done > gpurun_out/r2_slab.log 2>&1
