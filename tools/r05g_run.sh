# Round 5: why bench.py --single-process --gpus 8 runs 92-98 k when tools/slab_probe.py
# runs the same 8 slabs at 144-147 k: the clock probe and the twin board, toggled.
set -e
mkdir -p gpurun_out
O=gpurun_out/r05g_sp8_bench.jsonl
: > $O
for v in "default:" "noclock:--no-clock" "aged:--aged-board" "aged_noclock:--aged-board --no-clock"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 300 python3 bench.py --single-process --gpus 8 --no-secondary --no-cpu-baseline --steps 40 --warmup 5 $f > /tmp/sp8.json 2> /tmp/sp8.err
  python3 -c "import json,sys; d=json.load(open('/tmp/sp8.json')); print(json.dumps({'variant':sys.argv[1],'value':round(d['value']),'ms_per_step':round(d['ms_per_step'],3),'policy':d['config']['chunk_policy'],'mhz':(d.get('clock') or {}).get('sclk_mhz'),'verified':d['verified']}))" "$n" >> $O
  tail -1 $O
done
