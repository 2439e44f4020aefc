#!/bin/bash
# gpurun with waiting for a free box: retries ONLY while gpurun reports that
# nothing ran (exit 3 / transient: no slot or box free); any run that took a
# box returns its own status.   usage: tools/gwait.sh TIMEOUT 'command'
t=$1; shift
for i in $(seq 1 30); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1); rc=$?
  if echo "$out" | grep -q "status=transient"; then
    echo "[gwait] no box (try $i), waiting" >&2; sleep 100; continue
  fi
  echo "$out" | grep -v "every call"
  exit $rc
done
exit 3
