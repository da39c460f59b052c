# round 6 d: the driver's SCALE command at its defaults, rehearsed with the 8 ranks sharing this
# box's one GPU (RCCL under init_process_group("nccl")): 32^4 4a headline, 4b redistribution and
# the full 32^3 x 64 configs[4] chain with its whole-lattice single-GPU answers.  Device memory
# sampled every 10 s.
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
( while true; do date +%s >> $O/vram.log; rocm-smi --showmeminfo vram >> $O/vram.log 2>&1; sleep 10; done ) &
SMI=$!
SBX_BENCH_PROGRESS=1 timeout -k 10 1000 python3 bench.py --gpus 8 --share-gpu nccl > $O/scale8.json 2> $O/scale8_progress.log
rc=$?
kill $SMI
echo "rc=$rc" >> $O/scale8_progress.log
tail -5 $O/scale8_progress.log
cat $O/scale8.json
exit $rc
