cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
VARIANTS=0,7,8,9,10,11,12 LDS=0 timeout -k 10 400 python tools/bsr_sweep.py > gpurun_out/r2_bsr_sweep2.log 2>&1
