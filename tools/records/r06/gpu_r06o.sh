#!/bin/bash
# Round-6 lab: SwiGLU-backward dX with half the CUs started out of phase (CULLAVO_SWG_DELAY = s_sleep(127)
# count) -- per-shape bench per delay (one process each, the knob is read once), then steps alternating
set -o pipefail
TAG=${1:-r06o}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for dl in 0 2 4 6 8 12 0; do
  echo "delay $dl" >> $OUT/swg.txt
  CULLAVO_SWG_DELAY=$dl timeout -k 10 200 python -u tools/swiglu_dx_bench.py --rounds 3 >> $OUT/swg.txt 2>&1 || { tail -20 $OUT/swg.txt; exit 1; }
done
grep -v amdgpu.ids $OUT/swg.txt
bash tools/ab.sh $TAG/step 3 "d0=|" "d4=CULLAVO_SWG_DELAY=4|" "d8=CULLAVO_SWG_DELAY=8|"
