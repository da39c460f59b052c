# round 6 k: the driver's SCALE command at its defaults for N = 2 and 4 (ranks sharing the GPU)
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
for n in 2 4; do
  SBX_BENCH_PROGRESS=1 timeout -k 10 400 python3 bench.py --gpus $n --share-gpu nccl > $O/scale$n.json 2> $O/scale${n}_progress.log || { echo "N=$n failed"; tail -20 $O/scale${n}_progress.log; exit 1; }
  tail -c 600 $O/scale$n.json
done
