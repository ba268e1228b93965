# Round-end style GPU session: tests, full bench (with CPU baseline + recall), smoke, profiles.
# Every GPU step has its own time limit; the first failure ends the session.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread -rf > gpurun_out/t_all.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/t_all.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.log 2>&1; rb=$?
echo "bench rc=$rb"; tail -1 gpurun_out/bench_full.log
[ $rb -ne 0 ] && exit $rb
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rs=$?
echo "smoke rc=$rs"; tail -1 gpurun_out/smoke.log
[ $rs -ne 0 ] && exit $rs
[ "${NO_PROFILE:-0}" = 1 ] && exit 0
bash tools/profile.sh ${1:-r01}
