#!/bin/bash
# gpurun, retried only while the pool has no free slot or box (nothing ran, nothing charged)
out=$1; shift
for i in $(seq 1 24); do
  timeout 2400 /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  if grep -q "nothing was charged\|no free box right now\|backing off\|stopped responding while being prepared" $out && ! grep -q "status=ok" $out; then
    sleep 150; continue
  fi
  break
done
tail -80 $out
