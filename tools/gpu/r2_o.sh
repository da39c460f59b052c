cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 400 python tools/bsr_order.py natural blocked tile4 > gpurun_out/r2_bsr_colsplit.log 2>&1
