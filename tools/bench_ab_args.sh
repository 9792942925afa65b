#!/bin/bash
# Interleaved A/B of bench.py option sets on one box (the driver's measurement:
# headline on the seeded grid, aged board, config 4):
#   tools/bench_ab_args.sh <out.jsonl> <rounds> "<common args>" "<variant args>" ...
# Each variant is a string of extra bench.py arguments ("" = the defaults).
set -e
OUT=$1; ROUNDS=$2; ARGS=$3; shift 3
mkdir -p "$(dirname "$OUT")"
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    timeout -k 10 300 python bench.py $ARGS $v --no-secondary --no-cpu-baseline 2>/dev/null > /tmp/bench_ab_line.json
    python3 - "$v" "$r" >> "$OUT" <<'PY'
import json, sys
d = json.load(open("/tmp/bench_ab_line.json"))
a, c = d.get("aged_board") or {}, d.get("config4_1000gen") or {}
print(json.dumps({"variant": sys.argv[1] or "default", "round": int(sys.argv[2]), "value": round(d["value"], 1),
                  "mhz": (d.get("clock") or {}).get("sclk_mhz"), "step_ms": round(d["ms_per_step"], 4),
                  "policy": d["config"]["chunk_policy"], "split": d["config"].get("interior_split"),
                  "verified": d["verified"], "aged": round(a.get("value", 0), 1), "aged_mhz": a.get("sclk_mhz"),
                  "c4": round(c.get("value", 0), 1), "c4_mhz": c.get("sclk_mhz"), "c4_ok": c.get("verified")}))
PY
    tail -1 "$OUT"
  done
done
