# Round-5 measurement set at HEAD: tools/round_profile.sh (PMC + traces of the headline,
# bit k=1, byte k=32, byte k=1, default bench line, 8-slab rehearsal) and the k=8 wait-state pass.
set -e
export PYTHONUNBUFFERED=1
bash tools/round_profile.sh r05d
bash tools/pmc_waits.sh
