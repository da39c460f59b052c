# round 6 g: the 12x12 streaming BSR kernel (tests, chain-size and 16^4 timing)
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bsr.py -k "register_and_stream or 12x12 or stream_map" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
BLK=12 DT=cf DIMS=16,16,16,64 KINDS=stencil NCOLS=12 STREAMS=0,2:8:0,2:8:1,4:4:0,4:4:1,0,2:8:0,2:8:1,4:4:0,4:4:1 timeout -k 10 300 python -u tools/studies/bsr_bound.py > $O/bsr12_cf_chain.txt 2>&1 || { tail -20 $O/bsr12_cf_chain.txt; exit 1; }
cat $O/bsr12_cf_chain.txt
BLK=12 DT=cd L=16 KINDS=stencil NCOLS=12 STREAMS=0,2:4:0,2:4:1,0,2:4:0,2:4:1 timeout -k 10 300 python -u tools/studies/bsr_bound.py > $O/bsr12_cd.txt 2>&1 || { tail -20 $O/bsr12_cd.txt; exit 1; }
cat $O/bsr12_cd.txt
