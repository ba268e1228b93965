# Round-end style GPU session: tests, full bench (with CPU baseline + recall), profiles.
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -q -m gpu --timeout 300 -rf > gpurun_out/t_all.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/t_all.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2>&1; rb=$?
echo "bench rc=$rb"; tail -1 gpurun_out/bench_full.log
[ $rb -ne 0 ] && exit $rb
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/smoke.log
bash tools/profile.sh r01
