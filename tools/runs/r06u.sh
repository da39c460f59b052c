# round 6 u: eventless same-stream scratch reuse + region events in the bench: GPU suite, kernel
# timeline of the timed steps, the bench line
set -o pipefail
O=gpurun_out/r06u
mkdir -p $O
R=$(pwd)
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace -o run -- python3 $R/bench.py --no-side --no-cpu --steps 20 --warmup 10 > $R/$O/trace_bench.log 2>&1 || { tail -30 $R/$O/trace_bench.log; exit 1; }
cd $R
f=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python3 - "$f" > $O/timeline.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
g = [r for r in rows if "gemm_dma_kernel" in r["Kernel_Name"] or "splitk_reduce" in r["Kernel_Name"]]
prev = None
for r in g:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%8.1f gap %8.1f %s" % ((s - prev) / 1000 if prev else 0, (e - s) / 1000,
                                  "GEMM" if "gemm" in r["Kernel_Name"] else "reduce"))
    prev = e
PY
tail -24 $O/timeline.txt
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['shader_clock_GHz'], d['roofline']['kernel'])"
