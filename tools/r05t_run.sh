# Round 5: split cut fraction (runtime variants: the halves at 35/42/50/58 % of the interior).
set -e
bash tools/ab_libs.sh gpurun_out/r05t_cut_ab.jsonl 3 "--spec 8:d --spec 8:-1 --gens 400 --reps 2" base cut35 cut42 cut58
cat gpurun_out/r05t_cut_ab.jsonl
