#!/bin/bash
# LoRA dx kernel with 128-token tiles: LoRA tests, then the LoRA step (dx fusion on, off, on)
set -o pipefail
OUT=gpurun_out/r05x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_lora.py -x -q --timeout 300 --timeout-method thread > $OUT/lora_tests.log 2>&1
rc=$?; tail -3 $OUT/lora_tests.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0 1; do
  CULLAVO_LORA_DX_FUSE=$f timeout -k 10 400 python -u bench.py --trainable lora --no-sub --no-cpu-baseline --detail-out $OUT/lora_fuse$f.json > $OUT/lora_fuse$f.log 2>&1 || { tail -20 $OUT/lora_fuse$f.log; exit 1; }
  echo "fuse=$f"; python -c "import json; d=json.load(open('$OUT/lora_fuse$f.json')); print(d['value'], d['ms_per_step'])"
done
