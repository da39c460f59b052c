# round 6 b: the 8-site / 16-column BSR tile kernel (tests, timing, counters), the corrected
# streaming ceilings, the host-context detail device test
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bsr_tile.py tests/test_gpu_gemm.py -k "tile or host_context" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 120 tools/studies/stream_ceiling 2048 20 > $O/stream.txt 2>&1 || { cat $O/stream.txt; exit 1; }
cat $O/stream.txt
L=16 KINDS=stencil NCOLS=64 TILES=0,1,2,0,1,2 timeout -k 10 300 python -u tools/studies/bsr_bound.py > $O/bsr_tiles.txt 2>&1 || { tail -20 $O/bsr_tiles.txt; exit 1; }
cat $O/bsr_tiles.txt
timeout -k 10 300 bash tools/studies/pmc_bsr_tile.sh && cp -r gpurun_out/pmc_tile/summary.txt $O/pmc_summary.txt && cat $O/pmc_summary.txt
