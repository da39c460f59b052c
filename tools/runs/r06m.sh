# round 6 m: the reference's storage.cpp through the drop-in; refcaller tests
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_refcallers.py tests/test_gpu_storage.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
mkdir -p /tmp/sto && cd /tmp/sto && timeout -k 10 120 $GRAFT_REPO_ROOT/tests/refcallers/bin/storage > $GRAFT_REPO_ROOT/$O/storage_run.txt 2>&1; echo "rc=$?" >> $GRAFT_REPO_ROOT/$O/storage_run.txt
tail -12 $GRAFT_REPO_ROOT/$O/storage_run.txt
