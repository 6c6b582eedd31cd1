#!/bin/bash
# ViT bench line after naming the persistent forward family (gemm256p_k<MODE>) in bench.py
set -o pipefail
mkdir -p gpurun_out/r05vitname
timeout -k 10 400 python bench.py --workload vit --batch 64 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05vitname/vit.log 2>&1 || { tail -5 gpurun_out/r05vitname/vit.log; exit 1; }
tail -1 gpurun_out/r05vitname/vit.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['roofline'])[:600])"
echo all done
