# Round 4: guided chunk-rows per round rounded up (A/B).
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/ab_libs.sh gpurun_out/r04y_cpr_ab.jsonl 3 "--spec 8:d --gens 400 --reps 2" base cpru
cat gpurun_out/r04y_cpr_ab.jsonl
