#!/bin/bash
# usage: gpurun_retry.sh OUTFILE TIMEOUT 'command'   -- resubmits only when no box/slot was taken
out=$1; tmo=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $tmo -- "$cmd" > $out 2>&1
  rc=$?
  if grep -q "busy\|status=transient\|backing off\|stopped responding\|taken away" $out && ! grep -q "merged\|exit code\|rc=0\|rc=[1-9]" $out; then
    sleep 90; continue
  fi
  break
done
echo "done rc=$rc" >> $out
