mkdir -p gpurun_out/p
for pol in "PWR 500 FGD 500" "PWR" "BestFit" "FGD"; do
  for rm in 0 1; do
    [ "$pol" = "FGD" ] && [ $rm = 0 ] && rm=2
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --policy "$pol" --run-mode $rm > gpurun_out/p/b.json 2>gpurun_out/p/b.err || { cat gpurun_out/p/b.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/p/b.json'));print('$pol rm$rm', round(d['value']), round(d['ms_per_step'],2), d['roofline']['kernel'], d['roofline']['wgs_per_replica'])"
  done
done
for pol in "PWR 500 FGD 500" "PWR"; do
  KSIM_PROFILE=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --policy "$pol" --steps 1 --warmup 0 2>&1 >/dev/null | grep "ksim profile" || exit 1
done
