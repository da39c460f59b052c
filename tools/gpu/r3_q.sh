# round 3: config-2 GEMM forms (tools/gemm_memexp.hip)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_q && O=gpurun_out/r3_q &&
timeout -k 10 120 tools/gemm_memexp 20 > $O/gemm_memexp9.txt 2>&1
