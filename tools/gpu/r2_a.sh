cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 60 ./tools/mallocasync_repro > gpurun_out/r2_malloc.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 400 --timeout-method thread > gpurun_out/r2_gpu_tests.log 2>&1 ;
echo "pytest rc=$?" >> gpurun_out/r2_gpu_tests.log ;
timeout -k 10 400 python bench.py --steps 10 --warmup 5 > gpurun_out/r2_bench.log 2>&1 &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --share-gpu rccl --steps 3 --warmup 1 > gpurun_out/r2_share2_rccl.log 2>&1
