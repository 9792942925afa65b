# Round 4, folded tail strip (k=8 pair kernel, bytebit k>=20): parity first, then
# interleaved A/B of libgolhip variants (tools/build_variants.sh).
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 500 $T tests/test_gpu_parity.py -k "folded or k8 or bit_chunk or dead_goldens or bit_every or bytebit" > gpurun_out/r04n_fold_tests.log 2>&1
tail -1 gpurun_out/r04n_fold_tests.log
bash tools/ab_libs.sh gpurun_out/r04n_fold_ab.jsonl 3 "--spec 8:d --spec 8:-6 --gens 400 --reps 2" base nofold early1
cat gpurun_out/r04n_fold_ab.jsonl
bash tools/ab_libs.sh gpurun_out/r04n_bbfold_ab.jsonl 3 "--layout byte --spec 32:d --spec 28:d --gens 1024 --reps 2" base nofold bbch2
cat gpurun_out/r04n_bbfold_ab.jsonl
