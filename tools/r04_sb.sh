# Round 4: scheduling regions per event of the pair kernel with the early ring read (A/B).
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/ab_libs.sh gpurun_out/r04r_sb_ab.jsonl 3 "--spec 8:d --gens 400 --reps 2" base sb4 sb2
cat gpurun_out/r04r_sb_ab.jsonl
