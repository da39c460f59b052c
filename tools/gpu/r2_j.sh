cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 ./tools/gemm_tune 10 > gpurun_out/r2_gemm_tune.log 2>&1
