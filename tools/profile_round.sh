# Round profile of bench.py on the GPU box (run from the repo root through gpurun):
#   1. rocprofv3 --kernel-trace --stats  -> gpurun_out/prof/bench_results.db (+ the bench line)
#   2. rocprofv3 --pmc FETCH_SIZE         -> gpurun_out/pmc_fetch/  (separate pass)
#   3. rocprofv3 --pmc WRITE_SIZE         -> gpurun_out/pmc_write/  (separate pass)
# Summaries: tools/prof_summary.py and tools/pmc_summary.py (on the CPU side).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --no-cpu > $R/gpurun_out/prof_bench.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $R/gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $R/gpurun_out/pmc_write.log 2>&1
