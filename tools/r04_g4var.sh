set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/ab_libs.sh gpurun_out/r04g_g4_variants_ab.jsonl 3 "--spec 8:d --spec 8:-6 --gens 400 --reps 2" base sb2 sb4 sb8 nch2 nch2sb2
cat gpurun_out/r04g_g4_variants_ab.jsonl
