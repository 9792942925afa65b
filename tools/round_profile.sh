#!/bin/bash
# The round's measurement set on one MI355X (run from the repo root on the GPU box):
# PMC/trace passes of the headline, bit k=1, byte k=28 and byte k=1 configs, the default bench line,
# and the 8-slab single-process rehearsal of config 5 under a kernel trace.
#   tools/round_profile.sh <tag>
set -u
TAG=$1
R=$PWD
bash tools/profile.sh ${TAG}_k8 || exit 1
bash tools/profile.sh ${TAG}_k1 --no-cpu-baseline --no-secondary --no-aged --no-config4 -k 1 --steps 100 --warmup 3 --settle-s 0.3 || exit 1
bash tools/profile.sh ${TAG}_byte --no-cpu-baseline --no-secondary --no-aged --no-config4 --workload byte32768 --steps 36 --warmup 3 --settle-s 0.3 || exit 1
bash tools/profile.sh ${TAG}_byte1 --no-cpu-baseline --no-secondary --no-aged --no-config4 --workload byte32768 -k 1 --steps 100 --warmup 3 --settle-s 0.3 || exit 1
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_sp8 -o run -- \
  python3 $R/bench.py --single-process --gpus 8 --no-secondary --no-cpu-baseline --no-clock > $R/gpurun_out/${TAG}_bench_sp8.json \
  2> $R/gpurun_out/${TAG}_bench_sp8.err || exit 1
echo "round profile $TAG done"
