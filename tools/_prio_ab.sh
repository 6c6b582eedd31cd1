# A/B: training step on a high-priority stream vs the default stream (same box, alternating)
set -e
mkdir -p gpurun_out/prio
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/prio/base_$i.log 2>&1
  timeout -k 10 300 python bench.py --no-cpu-baseline --high-prio > gpurun_out/prio/prio_$i.log 2>&1
done
for f in gpurun_out/prio/*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
