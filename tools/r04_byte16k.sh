set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/ab_libs.sh gpurun_out/r04i_byte16k_ab.jsonl 2 "--layout byte --n 16384 --spec 28:d --spec 28:-2 --spec 28:110 --spec 28:150 --spec 28:200 --spec 24:d --spec 20:d --spec 16:d --spec 32:d --gens 1008 --reps 2" base rot2
cat gpurun_out/r04i_byte16k_ab.jsonl
