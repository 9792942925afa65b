set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/ab_libs.sh gpurun_out/r04l_early_rd_ab.jsonl 4 "--spec 8:d --spec 8:-6 --gens 400 --reps 2" base early0
cat gpurun_out/r04l_early_rd_ab.jsonl
