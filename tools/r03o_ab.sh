set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune.py --layout byte --gens 400 --reps 2 --spec 1:16 --spec 1:64 --spec 1:256 --spec 1:-1 > gpurun_out/r03o_byte1_chunks.jsonl
cat gpurun_out/r03o_byte1_chunks.jsonl
tools/ab_libs.sh gpurun_out/r03o_bbnt_ab.jsonl 2 "--layout byte --gens 1008 --reps 2 --spec 28:d" base ntst ntld ntboth
cat gpurun_out/r03o_bbnt_ab.jsonl
