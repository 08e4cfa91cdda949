set -o pipefail
# configs[3] A/B of the one-segment-block LDS hand-off ("onepass_sb1" default vs 0), three alternating
# pairs on one box, after the one-pass tests (profiles/r06/ab_sb1).  Usage (GPU box, repo root): bash tools/ab_sb1.sh
mkdir -p gpurun_out/r06j
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_onepass.py -k "segment_block or shapes or stop_rule or reference_fixture or graph or refresh" > gpurun_out/r06j/pytest.txt 2>&1 || exit $?
for r in 1 2 3; do
  for v in -1 0; do
    timeout -k 10 200 python3 bench.py --config 3 --no-cpu --no-side-legs --windows 5 --onepass-sb1 $v > gpurun_out/r06j/c3_sb1${v}_$r.json 2> gpurun_out/r06j/c3_sb1${v}_$r.err || exit $?
  done
done
