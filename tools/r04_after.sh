# Round-4 HEAD evidence, second call: fuzz (every path, bit k=8/3/5, RCCL shim),
# the headline's kernel trace + PMC passes, and a same-box A/B of a 6-slot LDS ring.
set -e
export PYTHONUNBUFFERED=1
T=${1:-r04p}
SEED0=421 bash tools/r04_fuzz.sh $T
bash tools/profile.sh ${T}_k8
bash tools/ab_libs.sh gpurun_out/${T}_slots6_ab.jsonl 3 "--spec 8:d --gens 400 --reps 2" base nofold slots6
cat gpurun_out/${T}_slots6_ab.jsonl
