#!/bin/bash
# round-4 first GPU pass: the new guard / config-3-batch tests (without -x: every result), then
# the self-launched 2-rank gloo rehearsal of bench.py on the one GPU
set -o pipefail
OUT=gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_oob_guard.py tests/test_full_size.py::test_7b_decoder_layer_config3_batch8 \
  "tests/test_ops_gpu.py::test_attention_config3_batch8_sampled_heads" "tests/test_ops_gpu.py::test_gemm_288_rows_bitwise_vs_256" \
  -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" $OUT/tests.log | sed 's/ *\[.*%\]//' | tail -60
grep -E "^E .*(non-finite|max\|err)" $OUT/tests.log | sort | uniq | head -30
[ $rc -le 1 ] || exit $rc
CULLAVO_DIST_BACKEND=gloo timeout -k 10 420 python -u bench.py --gpus 2 --no-sub --steps 2 --warmup 1 --batch 4 \
  --no-cpu-baseline > $OUT/bench_dp2_selflaunch.json 2> $OUT/bench_dp2_selflaunch.err
rc2=$?
echo "dp2 rc $rc2"; tail -c 1500 $OUT/bench_dp2_selflaunch.json; tail -5 $OUT/bench_dp2_selflaunch.err
exit $rc2
