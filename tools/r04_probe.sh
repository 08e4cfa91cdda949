mkdir -p gpurun_out/r04_probe
timeout -k 10 60 tools/_cvt_rate_probe > gpurun_out/r04_probe/cvt_rate.txt 2>&1
