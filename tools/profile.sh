#!/bin/bash
# Kernel trace + PMC passes of bench.py on one MI355X (run on the GPU box from the repo root).
#   tools/profile.sh <tag> [bench args...]
# Writes rocprofv3 CSVs under gpurun_out/prof_<tag>_*; tools/pmc_summary.py condenses them.
# (--no-clock: counter collection serialises dispatches, and the clock probe
# runs beside the stencil launches until the host stops it.)
set -euo pipefail
TAG=${1:-r01}; shift || true
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--no-cpu-baseline --no-secondary --no-aged --no-config4 --steps 60 --warmup 3 --settle-s 0.5)
run() {   # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/prof_${TAG}_${name}" -o run -- \
    python3 "$REPO/bench.py" "${ARGS[@]}" --no-clock > "$OUT/prof_${TAG}_${name}.json" 2> "$OUT/prof_${TAG}_${name}.err"
}
run kt --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE
run cyc --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
echo "profile $TAG done"
