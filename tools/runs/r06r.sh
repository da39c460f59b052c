# round 6 r: streaming ceilings at the BSR kernels' own sizes (the working set of a repeated
# launch below 256 MB stays in the Infinity Cache, as it does for the BSR kernels' repeats)
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
for mib in 90 156 371 470 1586; do
  echo "== $mib MiB per buffer" >> $O/ceil.txt
  timeout -k 10 120 tools/studies/stream_ceiling $mib 40 >> $O/ceil.txt 2>&1 || { tail -20 $O/ceil.txt; exit 1; }
done
cat $O/ceil.txt
