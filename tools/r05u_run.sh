# Round 5: re-profile the headline at the -1 split default (per-step PMC record), then the full check.
set -e
bash tools/profile.sh r05u_k8split
python3 tools/pmc_summary.py gpurun_out prof_r05u_k8split > gpurun_out/r05u_k8split_pmc_summary.json
python3 tools/make_traffic.py gpurun_out prof_r05u_k8split bit131072_k8_split bit_pair_kernel --per-step 3
cp profiles/traffic.json gpurun_out/r05u_traffic.json
bash tools/final_check.sh r05u
