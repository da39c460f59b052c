cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out && R=$(pwd) &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_copy.py tests/test_gpu_golden.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2_copy_tests.log 2>&1 ;
timeout -k 10 120 ./tools/hipsparse_bsr > gpurun_out/r2_hipsparse.log 2>&1 &&
cd /tmp &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_bsr_fetch -o run -- python3 $R/tools/bsr_order.py > $R/gpurun_out/pmc_bsr_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/pmc_bsr_hit -o run -- python3 $R/tools/bsr_order.py > $R/gpurun_out/pmc_bsr_hit.log 2>&1
