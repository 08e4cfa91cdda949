set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_onepass.py -k "graph" > gpurun_out/r03b/pytest_graph.txt 2>&1 || { tail -30 gpurun_out/r03b/pytest_graph.txt; exit 1; }
tail -3 gpurun_out/r03b/pytest_graph.txt
for rep in 1 2; do
for gm in 8 64; do
timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 5 --graph-max $gm > gpurun_out/r03b/b20_g${gm}_$rep.json 2> gpurun_out/r03b/b20_g${gm}_$rep.err || exit 1
timeout -k 10 200 python bench.py --no-cpu --steps 256 --warmup 200 --graph-max $gm > gpurun_out/r03b/b256_g${gm}_$rep.json 2> gpurun_out/r03b/b256_g${gm}_$rep.err || exit 1
done
done
for f in gpurun_out/r03b/b*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f', round(d['value'],1), [round(w['s']*1e3,3) for w in d['config']['windows']])"; done
