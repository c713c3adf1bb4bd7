mkdir -p gpurun_out
for l in base lr2 ar2 lrar2 base lrar2; do
  if [ $l = base ]; then lib=numpyro_amd/_lib/libnumpyro_amd.so; else lib=build/ab/$l/libnumpyro_amd.so; fi
  timeout -k 10 120 python bench.py --chains 512 --configs none --no-cpu-baseline --lib $lib > gpurun_out/s512_$l.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(\"gpurun_out/s512_$l.log\").read().strip().splitlines()[-1]); print(\"$l 512\", round(d[\"value\"]), d[\"leapfrog_launches\"], round(d[\"ms_per_step\"],4), round(d[\"potential_ms_per_launch\"],4))"
done
for l in base lrar2; do
  if [ $l = base ]; then lib=numpyro_amd/_lib/libnumpyro_amd.so; else lib=build/ab/$l/libnumpyro_amd.so; fi
  timeout -k 10 200 python bench.py --configs none --no-cpu-baseline --steps 50 --lib $lib > gpurun_out/s4096_$l.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(\"gpurun_out/s4096_$l.log\").read().strip().splitlines()[-1]); print(\"$l 4096\", round(d[\"value\"]), d[\"leapfrog_launches\"], round(d[\"ms_per_step\"],4), round(d[\"potential_ms_per_launch\"],4))"
done
