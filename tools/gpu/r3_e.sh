# round 3: shared-GPU rehearsals of the N>1 bench at the default sizes, with the answer checks
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_e &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --share-gpu rccl --steps 3 --warmup 1 > gpurun_out/r3_e/n2.json 2> gpurun_out/r3_e/n2.err &&
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --share-gpu rccl --steps 2 --warmup 1 > gpurun_out/r3_e/n4.json 2> gpurun_out/r3_e/n4.err &&
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29535 bench.py --share-gpu rccl --steps 2 --warmup 1 > gpurun_out/r3_e/n8.json 2> gpurun_out/r3_e/n8.err
