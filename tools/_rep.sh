mkdir -p gpurun_out
for lib in rossby-wave-ray-tracing_amd/librwrt_w1g6.so rossby-wave-ray-tracing_amd/librwrt_w2g2.so; do
 for rep in 1 2 4; do
  timeout -k 10 300 python bench.py --days 20 --steps 2 --warmup 1 --no-cpu --lib $lib --replicate $rep >> gpurun_out/rep.jsonl 2>>gpurun_out/rep.err || exit 1
 done
done
