set -e
for v in base nts ntl ntb; do
  if [ $v = base ]; then L=mpi_amd/libgolhip.so; else L=mpi_amd/libgolhip_$v.so; fi
  GOL_LIB=$L timeout -k 10 120 python tools/tune.py --ks 1,2,4 --wpls 4 --chunks=16,32 --reps 3 | sed "s/^/{\"v\":\"$v\",/; s/,{/,/" >> gpurun_out/tune_nt.jsonl
  GOL_LIB=$L timeout -k 10 120 python tools/tune.py --ks 7,8 --wpls 4 --chunks=-103,-104 --reps 3 | sed "s/^/{\"v\":\"$v\",/; s/,{/,/" >> gpurun_out/tune_nt.jsonl
done
