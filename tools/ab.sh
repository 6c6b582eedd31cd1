#!/bin/bash
# Alternating A/B of bench.py variants on one GPU box (guide §5.4 rule 24: interleaved runs, one
# device). Each variant is "NAME=ENV_ASSIGNMENTS|BENCH_ARGS"; every round runs every variant once.
#   bash tools/ab.sh <tag> <rounds> "new=|" "old=CULLAVO_GEMM_GROUP=4|" "lora=|--trainable lora"
# Results: gpurun_out/<tag>/<name>_<round>.json and a value / ms-per-step table on stdout.
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    NAME=${v%%=*}; REST=${v#*=}; ENVS=${REST%%|*}; ARGS=${REST#*|}
    env $ENVS timeout -k 10 400 python bench.py --no-sub --no-cpu-baseline $ARGS > $OUT/${NAME}_$r.json 2> $OUT/${NAME}_$r.err \
      || { echo "variant $NAME failed"; tail -20 $OUT/${NAME}_$r.err; exit 1; }
  done
done
for f in $OUT/*.json; do
  echo "$(basename $f .json) $(tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
