#!/bin/bash
# Round-end check of the tree on one MI355X box (run from the repo root): every GPU test, smoke(),
# the driver's bench command (20 steps / 5 warm-up) and the default bench -> gpurun_out/final/
set -o pipefail
OUT=gpurun_out/final
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_20_5.json 2> $OUT/bench_20_5.err || { tail -20 $OUT/bench_20_5.err; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
for f in $OUT/bench_20_5.json $OUT/bench_default.json; do
  python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['value'],1), d['roofline']['frac'], d['cpu_baseline']['value'])"
done
