set -e
export PYTHONUNBUFFERED=1
bash tools/final_check.sh r05b
bash tools/profile.sh r05b_byte --no-cpu-baseline --no-secondary --no-aged --no-config4 --workload byte32768 --steps 36 --warmup 3 --settle-s 0.3
bash tools/profile.sh r05b_b16k --no-cpu-baseline --no-secondary --no-aged --no-config4 --workload byte32768 --rows 16384 --cols 16384 -k 28 --steps 40 --warmup 3 --settle-s 0.3
S=""; for k in 24 28 32; do for c in d -1 -2 48 64 96 128; do S="$S --spec $k:$c"; done; done
timeout -k 10 400 python tools/tune.py --layout byte --n 16384 $S --gens 1344 --reps 2 > gpurun_out/r05b_byte16k_sweep.jsonl
tail -3 gpurun_out/r05b_byte16k_sweep.jsonl
