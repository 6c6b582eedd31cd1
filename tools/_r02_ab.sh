set -o pipefail
mkdir -p gpurun_out/r02_ab
for m in 4 5 4 5; do
  CULLAVO_ATTN_BWD_MODE=$m timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/r02_ab/b$m.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/r02_ab/b$m.log').read().strip().splitlines()[-1]); print('mode $m', d['value'], d['ms_per_step'])"
done
