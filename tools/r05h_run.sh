# Round 5: the hardware-queue explanation of r05g, checked: 4 slabs (2 x 8 streams + the probe
# fit 24 queues) with and without the twin; 8 slabs at HEAD (twin skipped when it does not fit).
set -e
mkdir -p gpurun_out
O=gpurun_out/r05h_sp_bench.jsonl
: > $O
for v in "sp4_twin:--gpus 4" "sp4_aged:--gpus 4 --aged-board" "sp8_head:--gpus 8" "sp8_q32_twin_forced:--gpus 8"; do
  n=${v%%:*}; f=${v#*:}
  E=""
  [ "$n" = sp8_q32_twin_forced ] && E="GPU_MAX_HW_QUEUES=32"
  env $E timeout -k 10 300 python3 bench.py --single-process --no-secondary --no-cpu-baseline --steps 40 --warmup 5 $f > /tmp/sp.json 2> /tmp/sp.err
  python3 -c "import json,sys; d=json.load(open('/tmp/sp.json')); print(json.dumps({'variant':sys.argv[1],'value':round(d['value']),'ms_per_step':round(d['ms_per_step'],3),'mhz':(d.get('clock') or {}).get('sclk_mhz'),'board':d['board'][:60],'verified':d['verified']}))" "$n" >> $O
  tail -1 $O
done
