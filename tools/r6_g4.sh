set -o pipefail
mkdir -p gpurun_out/r6
for dt in f32 bf16; do
  timeout -k 10 200 python bench.py --dp on --steps 50 --warmup 10 --no-cpu-baseline --no-roofline --dtype $dt > gpurun_out/r6/dp_on_$dt.json 2> gpurun_out/r6/dp_on_$dt.log || exit 1
  cat gpurun_out/r6/dp_on_$dt.json
done
JR_BENCH_ONE_DEVICE=1 JR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/r6/rehearsal2.json 2> gpurun_out/r6/rehearsal2.log || exit 1
cat gpurun_out/r6/rehearsal2.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanes299.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r6/lanes.log 2>&1; echo pytest rc=$?
tail -8 gpurun_out/r6/lanes.log
