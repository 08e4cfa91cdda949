#!/bin/bash
# Round-2 profiles on the GPU box: rocprofv3 kernel trace + stats of the bench workloads
# (configs[1] default line, configs[3], configs[4], configs[2] on one GPU), then separate PMC
# passes (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md's HBM recipe) for the dominant kernels,
# and the per-launch traffic summary.  Usage (repo root, GPU box): tools/profile_r02.sh [TAG]
set -e
R=$(pwd)
TAG=${1:-r02}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
trace() {   # name, bench args
    local n=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$n -- \
        python3 $R/bench.py --no-cpu "$@" > $OUT/bench_$n.json 2> $OUT/trace_$n.err
}
pmc() {     # name, counter, regex, bench args
    local n=$1 c=$2 rx=$3; shift 3
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/${c}_$n --kernel-include-regex "$rx" -- \
        python3 $R/bench.py --no-cpu --steps 6 --warmup 2 --windows 1 --ramp 8 "$@" > $OUT/b_${c}_$n.json 2> $OUT/${c}_$n.err
}
if [ -z "$SKIP_TRACE" ]; then
trace c1
trace c3 --config 3
trace c4 --config 4
trace c2 --config 2 --steps 64 --warmup 40
fi
pmc c1 FETCH_SIZE "k_onepass<|k_onepass_tail" &&
pmc c1 WRITE_SIZE "k_onepass<|k_onepass_tail" &&
pmc c3 FETCH_SIZE "k_onepass<" --config 3 &&
pmc c3 WRITE_SIZE "k_onepass<" --config 3 &&
pmc c4 FETCH_SIZE "k_panel_pass" --config 4 &&
pmc c4 WRITE_SIZE "k_panel_pass" --config 4
cd $R
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
export PMC_OUT=$OUT/pmc_traffic.json
python3 tools/pmc_traffic.py $OUT/FETCH_SIZE_c1 $OUT/WRITE_SIZE_c1 m8192_n65536_b1_float_g1 $((8192*65536*4 + 8*8192 + 16*65536)) > /dev/null
python3 tools/pmc_traffic.py $OUT/FETCH_SIZE_c3 $OUT/WRITE_SIZE_c3 m1048576_n4096_b1_float_g1 $((1048576*4096*4 + 8*1048576 + 16*4096)) > /dev/null
python3 tools/pmc_traffic.py $OUT/FETCH_SIZE_c4 $OUT/WRITE_SIZE_c4 panel_m8192_n65536_k128 $((2*8192*65536 + 8*128*(8192+65536))) > /dev/null
echo done
