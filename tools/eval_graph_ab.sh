for r in 1 2; do for dt in bf16 f32; do for args in "--graph" ""; do
  out=$(timeout -k 10 150 python bench.py --mode eval --no-roofline --no-cpu-baseline --dtype $dt $args 2>&1); rc=$?
  echo "eval $dt [${args:-eager}] $(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1)"
  if [ $rc -ne 0 ]; then echo "$out" | tail -5; exit $rc; fi
done; done; done
