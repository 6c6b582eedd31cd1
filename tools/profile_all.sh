#!/bin/bash
# Per-workload round profiles (tools/profile_round.sh) for the bench workloads, then the merged PMC
# record file: bash tools/profile_all.sh <tag> [workload ...]   -> gpurun_out/<tag>/roofline_traffic.json
# (workloads: config3-full config3-lora config5-full config2-vit; default all four)
set -e
TAG=${1:-prof}; shift || true
WLS=${*:-config3-full config3-lora config5-full config2-vit}
for w in $WLS; do
  case $w in
    config3-full) bash tools/profile_round.sh $TAG/$w $w "gemm256_k<1, 1, 1, 256, 256, 1, false, false, 1>" ;;
    config3-lora) bash tools/profile_round.sh $TAG/$w $w "gemm256_k<0, 0, 1, 288, 256, 1, true, false, 0>" --trainable lora ;;
    config5-full) bash tools/profile_round.sh $TAG/$w $w "gemm256_k<1, 1, 1, 256, 256, 1, false, false, 1>" --config llava-1.5-13b --batch 4 --text-len 1025 ;;
    config2-vit) bash tools/profile_round.sh $TAG/$w $w "gemm256pd_k<*, 256>" --workload vit --batch 64 ;;
    *) echo "unknown workload $w"; exit 1 ;;
  esac
done
python - "$TAG" $WLS <<'PY'
import json, sys
tag = sys.argv[1]
recs = []
for w in sys.argv[2:]:
    r = json.load(open(f"gpurun_out/{tag}/{w}/roofline_traffic.json"))
    recs += r if isinstance(r, list) else [r]
note = ("PMC records per (workload, kernel): rocprofv3 --pmc passes of bench.py --no-sub on that workload "
        "(tools/profile_round.sh); bytes_per_launch = 2 x FETCH_SIZE (gfx950 wide-read correction) + WRITE_SIZE")
json.dump({"note": note, "records": recs}, open(f"gpurun_out/{tag}/roofline_traffic.json", "w"), indent=1)
PY
echo all done
