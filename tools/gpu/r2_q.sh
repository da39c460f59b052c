cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python tools/bsr_probe.py > gpurun_out/r2_bsr_probe.log 2>&1 &&
VARIANTS=0,13,14,15 LDS=0,24576 timeout -k 10 300 python tools/bsr_sweep.py > gpurun_out/r2_bsr_sweep3.log 2>&1
