set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=""
for c in -1 -2 -3 -4 -6 -8 -102 -103 -104 -105 -106 256 368 512; do S="$S --spec 8:$c"; done
timeout -k 10 600 python tools/tune.py $S --gens 400 --reps 3 > gpurun_out/r04d_g4_policy_sweep.jsonl
cat gpurun_out/r04d_g4_policy_sweep.jsonl
