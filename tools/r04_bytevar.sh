set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/ab_libs.sh gpurun_out/r04h_byte_rot2_ab.jsonl 3 "--layout byte --spec 28:d --spec 32:d --spec 24:d --gens 1008 --reps 2" base rot2
cat gpurun_out/r04h_byte_rot2_ab.jsonl
