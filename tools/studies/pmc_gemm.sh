# MFMA utilisation counters of the GEMM kernel (tools/studies/gemm_tune, ONLY=a); run on the GPU box
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/gpmc
export ONLY=a
for c in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/gpmc/$n -o run -- $R/tools/studies/gemm_tune 3 > /dev/null 2>&1
done
for f in $(find $R/gpurun_out/gpmc -name "*counter_collection.csv"); do python3 - "$f" <<'PY'
import csv,sys,collections
agg=collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "gemm_dma_kernel" in r["Kernel_Name"] and "8, 4, 2, false" in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k,v in agg.items(): print(k, sum(v)/len(v), len(v))
PY
done
