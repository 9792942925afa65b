# Round 5: parity of the pair-kernel variants (alive plane in LDS, mid-event ring prefetch),
# then interleaved same-box A/B (tools/tune.py, then the driver's bench shape).
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
for v in bcl pf2 pf4 pf6; do
  GOL_LIB=mpi_amd/libgolhip_$v.so timeout -k 10 400 $T tests/test_gpu_parity.py -k "k8 or folded or dead_goldens or bit_chunk or mesh_goldens or serial_goldens" > gpurun_out/r05c_${v}_tests.log 2>&1
  tail -1 gpurun_out/r05c_${v}_tests.log
done
bash tools/ab_libs.sh gpurun_out/r05c_pair_ab.jsonl 3 "--spec 8:d --gens 400 --reps 2" base bcl pf2 pf4 pf6
cat gpurun_out/r05c_pair_ab.jsonl
bash tools/bench_ab.sh gpurun_out/r05c_pair_bench_ab.jsonl 2 "--steps 20 --warmup 5 --no-config4" base pf2 pf4 bcl
