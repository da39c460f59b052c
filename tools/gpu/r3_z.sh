# round 3: block transpose with line-aligned tiles -- copy tests, copy kinds, FETCH_SIZE / WRITE_SIZE of the copy kernels
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_z && O=$(pwd)/gpurun_out/r3_z && R=$(pwd) &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_copy_trans.py tests/test_gpu_copy.py tests/test_gpu_golden.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
COPY_KINDS=1 SBX_COPY_DEBUG=1 timeout -k 10 300 python tools/copy_shapes.py > $O/copy_kinds.txt 2> $O/copy_kinds.err &&
cd /tmp &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/tools/copy_shapes.py > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/tools/copy_shapes.py > $O/pmc_write.log 2>&1
