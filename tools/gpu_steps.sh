#!/bin/bash
# A GPU-box pass of named steps, each under its own time limit, logs under gpurun_out/<tag>/:
#   gpurun -- bash tools/gpu_steps.sh <tag> <step> [<step> ...]
# step = name:seconds:command (the command runs under bash -c).  A step that exits 0 or 1 (pytest's
# "tests failed") lets the pass go on; any other status (a time limit 124/137, an abort 134, a
# segfault 139, a Python crash) ends the pass there: nothing else is started on the GPU after it.
set -uo pipefail
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p "$O"
for spec in "$@"; do
  name=${spec%%:*}
  rest=${spec#*:}
  secs=${rest%%:*}
  cmd=${rest#*:}
  echo "[$name] start $(date +%T)"
  timeout -k 10 "$secs" bash -c "$cmd" > "$O/$name.log" 2>&1
  rc=$?
  echo "[$name] rc=$rc $(date +%T)"
  tail -3 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[$name] stopping the pass (rc=$rc)"
    exit $rc
  fi
done
