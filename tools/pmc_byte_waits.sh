#!/bin/bash
# Wait-state PMC passes of the byte-board bytebit kernel at k = 20 and k = 28
# (is it memory- or issue-bound?).  Run on the GPU box from the repo root:
#   tools/pmc_byte_waits.sh <tag>
set -euo pipefail
TAG=${1:-byte}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
for k in 20 28; do
  A=(--no-cpu-baseline --no-secondary --no-fresh --no-clock --workload byte32768 -k $k --steps $((1008 / k)) --warmup 3 --settle-s 0.3)
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d "$OUT/prof_${TAG}_k${k}_waits" -o run -- \
    python3 "$REPO/bench.py" "${A[@]}" > "$OUT/prof_${TAG}_k${k}_waits.json" 2> "$OUT/prof_${TAG}_k${k}_waits.err"
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv \
    -d "$OUT/prof_${TAG}_k${k}_waits2" -o run -- \
    python3 "$REPO/bench.py" "${A[@]}" > "$OUT/prof_${TAG}_k${k}_waits2.json" 2> "$OUT/prof_${TAG}_k${k}_waits2.err"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_k${k}_kt" -o run -- \
    python3 "$REPO/bench.py" "${A[@]}" > "$OUT/prof_${TAG}_k${k}_kt.json" 2> "$OUT/prof_${TAG}_k${k}_kt.err"
done
echo "byte waits $TAG done"
