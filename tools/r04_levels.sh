# Round 4: warm-up levels of the byte kernel at k = 32 (A/B of libgolhip variants).
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/ab_libs.sh gpurun_out/r04x_bb_levels_ab.jsonl 3 "--layout byte --spec 32:d --gens 1024 --reps 2" base lv2 lv6 lv8
cat gpurun_out/r04x_bb_levels_ab.jsonl
