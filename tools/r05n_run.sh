# Round 5: split interior default — full check, then an interleaved same-box
# A/B of the driver's bench command: split (default) vs unsplit.
set -e
bash tools/final_check.sh r05n
bash tools/bench_ab_args.sh gpurun_out/r05n_split_ab.jsonl 3 "--gpus 1" "" "--interior-split 1"
# multi-slab (the N>1 rank shape: boundary bands + halo exchange per slab), split vs unsplit
timeout -k 10 400 python tools/slab_probe.py --slabs 1,2,4 --spec 1:d:2 --spec 1:d:1 --reps 2 > gpurun_out/r05n_slab_split.jsonl
cat gpurun_out/r05n_slab_split.jsonl
