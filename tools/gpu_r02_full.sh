# one GPU call: the whole -m gpu suite, smoke(), the default bench, and the round's rocprof passes
# (10M headline + the 1.25M shard of an 8-way split).  Usage on the GPU box: bash tools/gpu_r02_full.sh <tag>
set -e
TAG=${1:-r02}
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_$TAG.log 2>&1
timeout -k 10 600 python -u bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err
bash tools/profile.sh ${TAG}_10M
bash tools/profile.sh ${TAG}_shard1.25M --rows 1250000 --steps 20 --warmup 3 --no-cpu
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 50 --warmup 5 --no-cpu > $O/bench_${TAG}_shard1.25M.json 2>&1
