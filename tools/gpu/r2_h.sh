cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_bsr.py tests/test_gpu_golden.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2_bsr_tests.log 2>&1 &&
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --share-gpu rccl --steps 3 --warmup 1 > gpurun_out/r2_share2_rccl_b.log 2>&1
