# round 6 t: kernel timeline of the bench's timed contraction steps (no side measurements)
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/$O/trace -o run -- python3 $R/bench.py --no-side --steps 20 --warmup 10 > $R/$O/bench.log 2>&1 || { tail -30 $R/$O/bench.log; exit 1; }
cd $R
f=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python3 - "$f" > $O/timeline.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = rows[-40:]
prev = None
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0
    print("%9.1f us gap  %9.1f us  %s" % (gap, (e - s) / 1000, r["Kernel_Name"][:110]))
    prev = e
PY
cat $O/timeline.txt
m=$(find $O/trace -name '*memory_copy_trace.csv' | head -1)
[ -n "$m" ] && wc -l "$m"
tail -2 $O/bench.log | cut -c1-300
