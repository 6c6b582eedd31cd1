#!/bin/bash
# one-box A/B of the library before the round-5 epilogue work (tools/lab/bin/libcullavo_old.so, built
# from commit 9abe03e) against the current in-tree library: the default bench, alternating
set -o pipefail
OUT=gpurun_out/r05ae
mkdir -p $OUT
export TMPDIR=/tmp
for v in new old new old; do
  if [ $v = old ]; then export CULLAVO_LIB_AB=$PWD/tools/lab/bin/libcullavo_old.so; else unset CULLAVO_LIB_AB; fi
  timeout -k 10 600 python -u bench.py --no-cpu-baseline --detail-out $OUT/bench_$v.json > $OUT/bench_$v.log 2>&1 || { tail -20 $OUT/bench_$v.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$v.json')); print('$v', d['value'], d['ms_per_step'], ' '.join(f'{k}={v[\"value\"]}' for k,v in d['workloads'].items()))"
done
