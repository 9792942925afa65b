# Round-4 HEAD check on one MI355X: full -m gpu suite, smoke, the driver's bench command,
# then a same-box A/B of the new pair-kernel defaults (fold + early ring read) against each off.
set -e
export PYTHONUNBUFFERED=1
bash tools/final_check.sh ${1:-r04o}
bash tools/ab_libs.sh gpurun_out/${1:-r04o}_defaults_ab.jsonl 2 "--spec 8:d --gens 400 --reps 2" base nofold early0
cat gpurun_out/${1:-r04o}_defaults_ab.jsonl
