#!/bin/bash
# Wait-state PMC pass of the k=8 bit kernel (is it issue- or latency-bound?).
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
timeout -s KILL 120 rocprofv3 --list-avail > "$OUT/pmc_avail.txt" 2>&1 || true
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_WAVES \
  --output-format csv -d "$OUT/prof_waits" -o run -- python3 "$REPO/bench.py" --no-cpu-baseline --no-secondary --no-aged --no-config4 --no-clock --steps 20 --warmup 2 > "$OUT/prof_waits.json" 2> "$OUT/prof_waits.err"
echo done
