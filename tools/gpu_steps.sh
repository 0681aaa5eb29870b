#!/bin/bash
# Run GPU steps in order; stop at the first fault/abort/timeout (rc not in {0,1}).
# usage: tools/gpu_steps.sh "<name>:<timeout>:<cmd>" ...
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] timeout ${tmo}s: $cmd"
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc=$rc"; exit $rc; fi
done
