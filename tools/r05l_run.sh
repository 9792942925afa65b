# Round 5: the split interior, wider sweep (bit k=8 policies; byte k=32; small board).
set -e
mkdir -p gpurun_out
S=""; for c in -1 -2 -3 -4 -102 -103 256 368 512; do S="$S --spec 8:$c:2"; done
timeout -k 10 500 python tools/tune.py $S --spec 8:d:1 --spec 8:-3:1 --gens 400 --reps 3 > gpurun_out/r05l_bit_sweep.jsonl
cat gpurun_out/r05l_bit_sweep.jsonl
timeout -k 10 300 python tools/tune.py --layout byte --spec 32:d:1 --spec 32:d:2 --spec 32:-2:2 --spec 32:-3:2 --gens 1024 --reps 2 > gpurun_out/r05l_byte_sweep.jsonl
cat gpurun_out/r05l_byte_sweep.jsonl
timeout -k 10 300 python tools/tune.py --layout byte --n 16384 --spec 28:d:1 --spec 28:d:2 --spec 28:-2:2 --gens 1008 --reps 2 > gpurun_out/r05l_byte16k_sweep.jsonl
cat gpurun_out/r05l_byte16k_sweep.jsonl
