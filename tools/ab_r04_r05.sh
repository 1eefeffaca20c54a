cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for d in _abr04 .; do
    for dt in f32 bf16; do
      st=30; [ $dt = bf16 ] && st=60
      ms=$(cd $d && timeout -k 10 150 python bench.py --no-roofline --no-cpu-baseline --steps $st --warmup 5 --dtype $dt 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | head -1)
      echo "round $r [$d $dt] $ms"
    done
  done
done
