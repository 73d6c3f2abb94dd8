#!/bin/bash
# rocprofv3 passes of one command (kernel trace + stats, then one PMC pass per counter group, each
# its own run as MI355X_MICROARCH.md prescribes), outputs under OUT.
#   bash scripts/prof_cmd.sh OUT "counters;counters;..." python3 prog.py args...
set -e
OUT=$1; GROUPS_=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$OUT"
OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- "$@" > "$OUT/trace.log" 2>&1
echo trace-done
i=0
IFS=';' read -ra G <<< "$GROUPS_"
for g in "${G[@]}"; do
    i=$((i + 1))
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $g -d "$OUT/pmc$i" -o run --output-format csv -- "$@" > "$OUT/pmc$i.log" 2>&1
    echo "pmc$i-done ($g)"
done
