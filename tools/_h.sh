mkdir -p gpurun_out/r02h
timeout -k 10 300 python3 bench.py > gpurun_out/r02h/bench_default.json 2> gpurun_out/r02h/bench_default.err &&
timeout -k 10 300 python3 bench.py --config 4 --no-cpu > gpurun_out/r02h/bench_c4.json 2> gpurun_out/r02h/bench_c4.err
