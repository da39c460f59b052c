# round 6 af: the driver's SCALE command at its defaults on the final tree (ranks sharing the
# box's GPU): N = 2, 4, 8
set -o pipefail
O=gpurun_out/r06af
mkdir -p $O
for n in 2 4 8; do
  SBX_BENCH_PROGRESS=1 timeout -k 10 400 python3 bench.py --gpus $n --share-gpu nccl > $O/scale$n.json 2> $O/scale${n}_progress.log || { echo "N=$n failed"; tail -20 $O/scale${n}_progress.log; exit 1; }
  python3 -c "
import json; d = json.loads(open('$O/scale$n.json').read().strip().splitlines()[-1])
print($n, d['value'], d['ms_per_step'], d.get('scale_check_ok'), d.get('strong_scaling_vs_1gpu'), d.get('strong_scaling_vs_1gpu_4b'), d['roofline']['kernel'][-90:])"
done
