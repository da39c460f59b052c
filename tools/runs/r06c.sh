# round 6 c: the 12x12 values-in-registers BSR kernel (tests, chain-size timing), DMA stream forms
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bsr.py -k "values_in_registers or 12x12" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 120 tools/studies/stream_ceiling 2048 20 > $O/stream.txt 2>&1 || { cat $O/stream.txt; exit 1; }
tail -5 $O/stream.txt
BLK=12 DT=cf DIMS=16,16,16,64 KINDS=stencil,self NCOLS=12 VREGS=0,1,2,3,0,1,2,3 timeout -k 10 300 python -u tools/studies/bsr_bound.py > $O/bsr12_cf_chain.txt 2>&1 || { tail -20 $O/bsr12_cf_chain.txt; exit 1; }
cat $O/bsr12_cf_chain.txt
BLK=12 DT=cd L=16 KINDS=stencil NCOLS=12 VREGS=0,1,2,3,0,1,2,3 timeout -k 10 300 python -u tools/studies/bsr_bound.py > $O/bsr12_cd.txt 2>&1 || { tail -20 $O/bsr12_cd.txt; exit 1; }
cat $O/bsr12_cd.txt
