#!/bin/bash
# Development GPU session: bash tools/gpu_session.sh <out dir> "<step name>|<seconds>|<command>" ...
# Each step runs under its own time limit, output to <out dir>/<name>.log.  Continues after a
# step that exits 0 or 1 (test failures); stops at anything else (fault, abort, time limit).
set -u
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  t0=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc $(( $(date +%s) - t0 ))s"; tail -4 "$OUT/$name.log" | cut -c1-600
  if [ $rc -gt 1 ]; then echo "stopping after $name"; exit $rc; fi
done
