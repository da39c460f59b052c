# round 6 n: storage_details.cpp through the drop-in
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_refcallers.py -k "storage" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
