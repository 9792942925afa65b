# Round 5: the split interior as the k = 8 default — the per-step PMC passes of
# the headline first (traffic.json's bit131072_k8_split, which bench.py's line
# and the contract test read), then the full -m gpu suite, smoke, the driver's
# bench command.
set -e
bash tools/profile.sh r05m_k8split
python3 tools/pmc_summary.py gpurun_out prof_r05m_k8split > gpurun_out/r05m_k8split_pmc_summary.json
python3 tools/make_traffic.py gpurun_out prof_r05m_k8split bit131072_k8_split bit_pair_kernel --per-step 3
cp profiles/traffic.json gpurun_out/r05m_traffic.json
bash tools/final_check.sh r05m
