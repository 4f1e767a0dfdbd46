# Round-6 final evidence, the other configs (r06_f4x): C2, C4, textured C3 / C4, the driver's 20-frame command
OUT=gpurun_out/r06_f4x; mkdir -p $OUT
for a in "C2:color" "C4:color" "C3:textured" "C4:textured"; do
  IFS=: read cfg sh <<< "$a"
  timeout -k 10 300 python bench.py --config $cfg --shading $sh --cpu-seconds 0 > $OUT/bench_${cfg}_${sh}.log 2>&1 || exit 1
  echo "$cfg $sh $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_${cfg}_${sh}.log) $(grep -o '"frame_latency_ms": [0-9.]*' $OUT/bench_${cfg}_${sh}.log) $(grep -o '"sync_frame_kernel_ms": [0-9.]*' $OUT/bench_${cfg}_${sh}.log) $(grep -o '"verified": [a-z]*' $OUT/bench_${cfg}_${sh}.log | head -1)"
done
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/drv_$i.log 2>&1 || exit 1
  echo "drv $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/drv_$i.log) $(grep -o '"verified": [a-z]*' $OUT/drv_$i.log | head -1)"
done
