#!/bin/bash
# Run GPU steps in order; stop at the first one that timed out / crashed (124, 137, 134, 139)
# so nothing else touches the GPU after a fault.  Usage: tools/gpu_step.sh "<name>|<seconds>|<cmd>" ...
mkdir -p gpurun_out
for spec in "$@"; do
    name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
    echo "== $name ($secs s): $cmd"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
    case $rc in 124|137|134|139) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
done
