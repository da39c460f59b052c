cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
PROBE=1 timeout -k 10 120 ./tools/gemm_tune > gpurun_out/r2_gemm_probe.log 2>&1
