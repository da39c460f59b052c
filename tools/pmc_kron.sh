# PMC counters of the Kronecker BSR kernel (tools/kron_bench.py, complex<double>, n = 12); run on the GPU box
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/kpmc
export KRON_ONLY=complex128:12
for c in "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/kpmc/$n -o run -- python3 $R/tools/kron_bench.py > /dev/null 2>&1
done
for f in $(find $R/gpurun_out/kpmc -name "*counter_collection.csv"); do python3 - "$f" <<'PY'
import csv,sys,collections
agg=collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "kron_lds" in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k,v in agg.items(): print(k, sum(v)/len(v), len(v))
PY
done
