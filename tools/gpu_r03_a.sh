# round 3, first GPU call: the GPU suite with the round's host changes, the driver-shaped bench, a
# rocprofv3 kernel trace of that exact bench command (+ PMC passes), and the N > 1 launcher on a
# one-GPU box (must fail loudly; the rehearsal with both ranks on GPU 0 must print n_gpus 2).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json; [ $rc -ne 0 ] && exit $rc
bash tools/profile.sh r03_10M --gpus 1 --steps 20 --warmup 5 || exit 1
python3 tools/summarize_profile.py gpurun_out/prof_r03_10M r03_10Mx1024_b64 20480000000 > /dev/null || exit 1
mkdir -p $O/profiles && cp profiles/r03_10Mx1024_b64_* $O/profiles/
timeout -k 10 180 python -u bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu > $O/gpus2.out 2> $O/gpus2.err
echo "gpus2 (expected to fail on a one-GPU box) rc=$?" | tee -a $O/gpus2.out
HIPRAG_BENCH_REHEARSE=1 timeout -k 10 300 python -u bench.py --gpus 2 --rows 2500000 --steps 20 --warmup 5 --recall-queries 4 > $O/rehearse2.json 2> $O/rehearse2.err
echo "rehearse rc=$?"; cat $O/rehearse2.json
