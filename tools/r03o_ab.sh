set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune.py --layout byte --gens 400 --reps 2 --spec 1:16 --spec 1:-1 --spec 1:-104 --spec 1:-102 --spec 1:-8 > gpurun_out/r03o_byte1_policies.jsonl
cat gpurun_out/r03o_byte1_policies.jsonl
timeout -k 10 300 python tools/tune.py --layout byte --gens 1008 --reps 2 --spec 28:-1 --spec 28:-2 --spec 28:-102 --spec 28:-104 --spec 28:400 > gpurun_out/r03o_byte28_policies.jsonl
cat gpurun_out/r03o_byte28_policies.jsonl
