# Round-4 final HEAD check: full -m gpu suite, smoke, the driver's bench command, fuzz.
set -e
export PYTHONUNBUFFERED=1
bash tools/final_check.sh ${1:-r04s}
SEED0=431 bash tools/r04_fuzz.sh ${1:-r04s}
