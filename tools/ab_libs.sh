#!/bin/bash
# A/B of libgolhip variant builds on the GPU box (run from the repo root):
#   tools/ab_libs.sh <out.jsonl> <rounds> "<tune.py args>" lib...   (lib: base = libgolhip.so, else libgolhip_<lib>.so)
# Rounds interleave the libraries so box drift hits all of them alike.
set -e
OUT=$1; ROUNDS=$2; ARGS=$3; shift 3
mkdir -p "$(dirname "$OUT")"
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    if [ "$v" = base ]; then L=mpi_amd/libgolhip.so; else L=mpi_amd/libgolhip_$v.so; fi
    GOL_LIB=$L timeout -k 10 200 python tools/tune.py $ARGS 2>/dev/null | sed "s/^{/{\"lib\":\"$v\",\"round\":$r,/" >> "$OUT"
  done
done
