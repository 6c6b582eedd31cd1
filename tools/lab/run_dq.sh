#!/bin/bash
# GPU box: the dQ ring lab (tools/lab/dq_lab.py)
set -o pipefail
OUT=gpurun_out/${1:-dq}
mkdir -p $OUT
timeout -k 10 300 python -u tools/lab/dq_lab.py --rounds 3 > $OUT/lab.txt 2>&1
rc=$?
grep -v amdgpu.ids $OUT/lab.txt | tail -24
exit $rc
