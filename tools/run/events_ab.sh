# what recording HIP events inside the timed region costs (config 2 headline step, 20/5 steps = the driver's shape)
for ev in 1 4 0 1 4 0; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --event-stride $ev > gpurun_out/ev_$ev.json 2>gpurun_out/ev_$ev.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ev_$ev.json'));print('event stride $ev', round(d['value']), 'ms/step', round(d['ms_per_step']*1e3,1), 'unproject', d['roofline']['launch_ms'], 'softargmax', d['softargmax_ms'])"
done
