cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python tools/bsr_order.py natural morton tile4 > gpurun_out/r2_bsr_order2.log 2>&1
