# GPU check used during development: parity tests, then quick benches (each step time-limited).
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -q -m gpu --timeout 300 -rf > gpurun_out/t1.log 2>&1; rc=$?
echo "pytest rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --rows 1000000 --dim 768 --steps 10 --warmup 2 --no-cpu > gpurun_out/b1.log 2>&1; rb=$?
  echo "bench1 rc=$rb"
  if [ $rb -eq 0 ]; then
    timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b2.log 2>&1; echo "bench2 rc=$?"
  fi
fi
tail -15 gpurun_out/t1.log; tail -3 gpurun_out/b1.log; tail -3 gpurun_out/b2.log
