cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --share-gpu rccl --steps 2 --warmup 1 --skip redistribution > gpurun_out/r2_share4_rccl.log 2>&1 &&
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --share-gpu rccl --steps 2 --warmup 1 --skip redistribution > gpurun_out/r2_share8_rccl.log 2>&1 &&
bash tools/profile_round.sh
