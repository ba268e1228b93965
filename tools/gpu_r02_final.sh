# round-end evidence with the final code: rocprof passes for the 10M headline and the 1.25M shard,
# then the default bench (its traffic fields read the summaries these passes produce)
set -e
TAG=${1:-r02}
bash tools/profile.sh ${TAG}_10M
bash tools/profile.sh ${TAG}_shard1.25M --rows 1250000 --steps 20 --warmup 3 --no-cpu
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 300 --warmup 10 --no-cpu > gpurun_out/bench_${TAG}_shard1.25M.json 2>&1
