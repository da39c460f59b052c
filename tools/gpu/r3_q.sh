# round 3: config-2 GEMM with its code shifted by 0 / 4 / 8 / 12 bytes (instruction placement)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_q && O=gpurun_out/r3_q &&
timeout -k 10 120 tools/gemm_memexp 20 > $O/shift0.txt 2>&1 &&
timeout -k 10 120 tools/gemm_memexp_s1 20 > $O/shift1.txt 2>&1 &&
timeout -k 10 120 tools/gemm_memexp_s2 20 > $O/shift2.txt 2>&1 &&
timeout -k 10 120 tools/gemm_memexp_s3 20 > $O/shift3.txt 2>&1
