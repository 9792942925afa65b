# Round-5 HEAD check: -m gpu suite, smoke, driver bench command, fuzz set.
set -e
export PYTHONUNBUFFERED=1
bash tools/final_check.sh r05i
bash tools/fuzz_set.sh r05i 511
