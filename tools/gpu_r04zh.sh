#!/bin/bash
# AdamW: two grid-stride steps per trip (new) vs one (old), alternating libraries on one box
set -o pipefail
OUT=gpurun_out/r04zh
mkdir -p $OUT
D=causal-unified-language-vision_amd
for lib in new old new old; do
  cp $D/libcullavo_hip_$lib.so $D/libcullavo_hip.so
  echo -n "$lib: "; timeout -k 10 120 python -u tools/adamw_bench.py 2>&1 | grep adamw || exit 1
done | tee $OUT/ab.txt
cp $D/libcullavo_hip_new.so $D/libcullavo_hip.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests -k "adamw or optim" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; exit $rc
