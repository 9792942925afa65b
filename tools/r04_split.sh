# Round 4: the pair kernel's row checks only where a chunk needs them (prologue at the
# top edge, main loop at the bottom edge / column masks): parity, then same-box A/B.
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_scale.py -k "folded or k8 or bit_chunk or dead_goldens or bit_every or headline or serial_goldens or mesh" > gpurun_out/r04q_split_tests.log 2>&1
tail -1 gpurun_out/r04q_split_tests.log
bash tools/ab_libs.sh gpurun_out/r04q_split_ab.jsonl 3 "--spec 8:d --spec 8:-6 --gens 400 --reps 2" base nosplit
cat gpurun_out/r04q_split_ab.jsonl
