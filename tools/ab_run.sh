#!/bin/bash
# Same-box A/B of libbpgl variants (tools/build_ab.sh): for each round and each variant NAME in
# $VARIANTS: the k_onepass stamps (build_ab/NAME_st.so, if present) at the N = 8 strong row shard,
# and the bench lines of the strong shard (one-rank RCCL row leg) and of configs[1].
# usage: VARIANTS="base drain" ROUNDS=2 tools/ab_run.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/ab_run}
mkdir -p $OUT
B="python3 bench.py --no-cpu --no-side-legs"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    if [ -f build_ab/${v}_st.so ] && [ "$r" = 1 ]; then
      timeout -k 10 120 python3 tools/onepass_stamps.py build_ab/${v}_st.so 1024 65536 --rows > $OUT/st_m1024_${v}.jsonl 2> $OUT/st_${v}.err || exit $?
      timeout -k 10 120 python3 tools/onepass_stamps.py build_ab/${v}_st.so 8192 65536 > $OUT/st_m8192_${v}.jsonl 2> $OUT/st8_${v}.err || exit $?
    fi
    BPGL_LIB=build_ab/$v.so timeout -k 10 200 $B --comm --shard rows --m 1024 --n-per-gpu 65536 --steps 256 --warmup 100 \
        --windows 5 > $OUT/m1024_${v}_$r.json 2> $OUT/m1024_${v}_$r.err || exit $?
    BPGL_LIB=build_ab/$v.so timeout -k 10 200 $B --steps 256 --warmup 100 --windows 5 ${EXTRA} > $OUT/c1_${v}_$r.json 2> $OUT/c1_${v}_$r.err || exit $?
    if [ -n "$C3" ]; then
      BPGL_LIB=build_ab/$v.so timeout -k 10 200 $B --config 3 --steps 64 --warmup 20 --windows 3 > $OUT/c3_${v}_$r.json 2> $OUT/c3_${v}_$r.err || exit $?
    fi
    if [ -n "$WEAK" ]; then
      BPGL_LIB=build_ab/$v.so timeout -k 10 200 $B --comm --shard rows --m 1024 --n-per-gpu 524288 --steps 256 --warmup 50 \
          --windows 3 > $OUT/m1024w_${v}_$r.json 2> $OUT/m1024w_${v}_$r.err || exit $?
    fi
  done
done
