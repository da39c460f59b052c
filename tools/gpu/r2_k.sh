cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
ONLY=w16 timeout -k 10 300 ./tools/gemm_tune 10 > gpurun_out/r2_gemm_tune2.log 2>&1
