# Round 5: multi-slab (the N>1 rank shape) under the split at each policy: -1 (default) vs -2 vs unsplit.
set -e
timeout -k 10 500 python tools/slab_probe.py --slabs 1,2,4 --spec 1:-1:2 --spec 1:-2:2 --spec 1:-3:2 --spec 1:d:1 --reps 2 > gpurun_out/r05v_slab_policy.jsonl
cat gpurun_out/r05v_slab_policy.jsonl
