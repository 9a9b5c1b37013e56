# Driver-shape vs settle vs 200-step bench runs of config 2, two each (profiles/r17_bench_shape.txt).
#   bash tools/shape_exp.sh   (on the GPU box; appends to gpurun_out/r17_shape_{a,b,c}.jsonl)
set -e
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python bench.py --config 2 --no-secondary --no-cpu-baseline --no-in-kernel-coords --steps 20 --warmup 5 >> gpurun_out/r17_shape_a.jsonl 2>/dev/null
  timeout -k 10 120 python bench.py --config 2 --no-secondary --no-cpu-baseline --no-in-kernel-coords --steps 20 --warmup 5 --settle 3 >> gpurun_out/r17_shape_b.jsonl 2>/dev/null
  timeout -k 10 120 python bench.py --config 2 --no-secondary --no-cpu-baseline --no-in-kernel-coords --steps 200 --warmup 5 >> gpurun_out/r17_shape_c.jsonl 2>/dev/null
done
