# Round 4: parity of the k=8 paths on a 2-word-group build (GOL_BIT_G4=0: the V=2 pair
# kernel) after the store-offset fix (the default build: r04u_default_tests.log).
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu"
GOL_LIB=mpi_amd/libgolhip_g2.so timeout -k 10 500 $T tests/test_gpu_parity.py -k "(folded or k8 or bit_chunk or dead_goldens or bit_every or serial_goldens or mesh_goldens) and not schedule_trial" > gpurun_out/r04u_g2_tests.log 2>&1
tail -1 gpurun_out/r04u_g2_tests.log
