#!/bin/bash
# In-kernel U fold (onepass_fold 1) against the separate k_onepass_fold / tail fold (0): the
# strong-scaling per-GPU row shapes through the one-rank RCCL leg, and one rank at configs[1] /
# configs[3] / the configs[2] per-GPU weak shape.  Usage (GPU box): tools/fold_sweep.sh
set -o pipefail
OUT=gpurun_out/fold_sweep
mkdir -p $OUT
run() {   # name, bench args...
    local name=$1; shift
    timeout -k 10 150 python3 bench.py --no-cpu --steps 256 --warmup 100 --windows 3 "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
}
for f in 0 1; do
  run rows_m1024_f$f --comm --shard rows --m 1024 --n-per-gpu 65536 --onepass-fold $f
  run rows_m2048_f$f --comm --shard rows --m 2048 --n-per-gpu 65536 --onepass-fold $f
  run rows_m4096_f$f --comm --shard rows --m 4096 --n-per-gpu 65536 --onepass-fold $f
  run rows_m1024_n524288_f$f --comm --shard rows --m 1024 --n-per-gpu 524288 --onepass-fold $f
  run one_c1_f$f --onepass-fold $f
done
run rows_m1024_c750_f1 --comm --shard rows --m 1024 --n-per-gpu 65536 --onepass-cache 750
