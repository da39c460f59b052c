cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python tools/bsr_timeline.py > gpurun_out/r2_timeline.log 2>&1
