#!/bin/bash
# the GPU suite minus the long full-size files, then smoke()
set -o pipefail
OUT=gpurun_out/r04_gpu
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests \
    --ignore=tests/test_longrun.py --ignore=tests/test_fullsize.py > $OUT/pytest_a.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
