set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/bench_ab.sh gpurun_out/r04c_g4_bench_ab.jsonl 3 "--steps 20 --warmup 5" base g2
bash tools/ab_libs.sh gpurun_out/r04c_g4_tune_ab.jsonl 2 "--spec 8:-6 --spec 8:-3 --spec 8:-103 --gens 400 --reps 2" base g2
cat gpurun_out/r04c_g4_tune_ab.jsonl
