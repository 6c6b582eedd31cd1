#!/bin/bash
# Per-workload round profiles (tools/profile_round.sh) for the four bench workloads, then the
# merged PMC record file: bash tools/profile_all.sh <tag>   -> gpurun_out/<tag>/roofline_traffic.json
set -e
TAG=${1:-prof}
bash tools/profile_round.sh $TAG/config3-full config3-full "gemm256_k<1, 1, 1, 256, 256, 1, false, false, 1>"
bash tools/profile_round.sh $TAG/config3-lora config3-lora "gemm256_k<0, 0, 1, 288, 256, 1, true, false, 0>" --trainable lora
bash tools/profile_round.sh $TAG/config5-full config5-full "gemm256_k<1, 1, 1, 256, 256, 1, false, false, 1>" --config llava-1.5-13b --batch 4 --text-len 1025
bash tools/profile_round.sh $TAG/config2-vit config2-vit "gemm256pd_k<*, 256>" --workload vit --batch 64
python - "$TAG" <<'PY'
import json, sys
tag = sys.argv[1]
recs = [json.load(open(f"gpurun_out/{tag}/{w}/roofline_traffic.json")) for w in ("config3-full", "config3-lora", "config5-full", "config2-vit")]
note = ("PMC records per (workload, kernel): rocprofv3 --pmc passes of bench.py --no-sub on that workload "
        "(tools/profile_round.sh); bytes_per_launch = 2 x FETCH_SIZE (gfx950 wide-read correction) + WRITE_SIZE")
json.dump({"note": note, "records": recs}, open(f"gpurun_out/{tag}/roofline_traffic.json", "w"), indent=1)
PY
echo all done
