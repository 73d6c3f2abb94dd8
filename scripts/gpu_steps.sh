#!/bin/bash
# Run GPU steps in order on the gpurun box, each under its own time limit. A step may fail its
# tests (pytest exit 1) and the next still runs; any other non-zero exit (abort, segfault, time
# limit, hang, internal error) ends the call there -- nothing more touches the GPU after it.
#   bash scripts/gpu_steps.sh OUTDIR "SECONDS CMD..." ["SECONDS CMD..." ...]
O=$1
shift
mkdir -p "$O"
i=0
for step in "$@"; do
    i=$((i + 1))
    secs=${step%% *}
    cmd=${step#* }
    echo "[step $i] $cmd"
    timeout -k 10 "$secs" bash -c "$cmd" > "$O/step$i.txt" 2>&1
    rc=$?
    echo "[step $i] rc=$rc"
    echo "$rc" > "$O/step$i.rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "[step $i] stopping: rc $rc"
        exit $rc
    fi
done
