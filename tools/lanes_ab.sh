for dt in bf16 f32; do
for args in "--graph" "--lanes 3" "" "--lanes 4" "--graph"; do
  out=$(timeout -k 10 150 python bench.py --no-roofline --no-cpu-baseline --dtype $dt $args 2>&1)
  rc=$?
  echo "$dt [$args] $(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1)"
  if [ $rc -ne 0 ]; then echo "$out" | tail -5; exit $rc; fi
done
done
