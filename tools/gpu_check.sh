#!/bin/bash
# One GPU-box pass: bench at the driver's 20/5 and at the default 256/200, smoke, then the GPU
# test suite.  Usage (repo root, on the box): tools/gpu_check.sh TAG [pytest args...]
set -o pipefail
TAG=${1:-check}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_20_5.json 2> $OUT/bench_20_5.err &&
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
exit $rc
