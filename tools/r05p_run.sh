# Round 5: split vs unsplit at the driver's own shape (--steps 20 --warmup 5), interleaved.
set -e
bash tools/bench_ab_args.sh gpurun_out/r05p_split_ab_driver.jsonl 4 "--gpus 1 --steps 20 --warmup 5" "" "--interior-split 1"
