set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for v in early1 clip1; do
  GOL_LIB=mpi_amd/libgolhip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "k8 or bit or dead or mesh" > gpurun_out/r04l_${v}_tests.log 2>&1
  tail -1 gpurun_out/r04l_${v}_tests.log
done
GOL_LIB=mpi_amd/libgolhip_bbch2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "bytebit" > gpurun_out/r04l_bbch2_tests.log 2>&1
tail -1 gpurun_out/r04l_bbch2_tests.log
bash tools/ab_libs.sh gpurun_out/r04l_clip_early_ab.jsonl 3 "--spec 8:d --spec 8:-6 --gens 400 --reps 2" base early1 clip1
cat gpurun_out/r04l_clip_early_ab.jsonl
bash tools/ab_libs.sh gpurun_out/r04l_bbch2_ab.jsonl 3 "--layout byte --spec 32:d --gens 1024 --reps 2" base bbch2
cat gpurun_out/r04l_bbch2_ab.jsonl
