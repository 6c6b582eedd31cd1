#!/bin/bash
# Round-6 lab: the SwiGLU-backward epilogue with every item's gate|up loads in flight at once per row half
# (gemm_common.h SWG_NB = 0, library built into tools/lab/so/ab/) against the default (4 items ahead)
set -o pipefail
TAG=${1:-r06nb}; OUT=gpurun_out/$TAG; mkdir -p $OUT
AB=tools/lab/so/ab/libcullavo_nb0.so
for r in 1 2; do
  timeout -k 10 200 python -u tools/swiglu_dx_bench.py --rounds 3 > $OUT/def_$r.txt 2>&1 || { tail -20 $OUT/def_$r.txt; exit 1; }
  CULLAVO_LIB_AB=$AB timeout -k 10 200 python -u tools/swiglu_dx_bench.py --rounds 3 > $OUT/nb0_$r.txt 2>&1 || { tail -20 $OUT/nb0_$r.txt; exit 1; }
done
for r in 1 2; do echo "default $r"; grep "swiglu_prefetch\|bitwise" $OUT/def_$r.txt; echo "nb0 $r"; grep "swiglu_prefetch\|bitwise" $OUT/nb0_$r.txt; done
bash tools/ab.sh $TAG/step 2 "c=|" "cnb0=CULLAVO_LIB_AB=$AB|"
