# SQ counters of the config-2 GEMM launch (tools/studies/gemm_one.py), one rocprofv3 pass per counter
# group (MI355X_MICROARCH.md: <= 8 SQ, <= 2 GRBM counters per pass); run on the GPU box:
#   bash tools/studies/pmc_gemm_counters.sh <tag>   (env LOADERS / SPREAD select the variant)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-base}
O=$R/gpurun_out/gpmc_$T
mkdir -p $O
i=0
for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAIT_INST_LDS" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/p$i -o run -- python3 $R/tools/studies/gemm_one.py > $O/p$i.log 2>&1 || echo "pass $i failed (see $O/p$i.log)"
done
python3 - $O <<'PY'
import csv, collections, glob, json, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm_dma_kernel" in r["Kernel_Name"] and "128, 128, 16, 4, 4" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: sum(v[2:]) / max(1, len(v[2:])) for k, v in agg.items()}
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1, sort_keys=True)
print(json.dumps(out, indent=1, sort_keys=True))
PY
