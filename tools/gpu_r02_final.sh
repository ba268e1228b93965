# round-end evidence with the final code, all on ONE box so the numbers agree: rocprof passes for the
# 10M headline and the 1.25M shard, their summaries (written into profiles/ here, where bench.py reads
# its traffic fields, and copied to gpurun_out/profiles_new/ to come back), then the default bench and
# the shard bench.
set -e
TAG=${1:-r02}
bash tools/profile.sh ${TAG}_10M
bash tools/profile.sh ${TAG}_shard1.25M --rows 1250000 --steps 20 --warmup 3 --no-cpu
python3 tools/summarize_profile.py gpurun_out/prof_${TAG}_10M ${TAG}_10Mx1024_b64 20480000000 > /dev/null
python3 tools/summarize_profile.py gpurun_out/prof_${TAG}_shard1.25M ${TAG}_shard1.25M_b64 2560000000 > /dev/null
mkdir -p gpurun_out/profiles_new
cp profiles/${TAG}_10Mx1024_b64_* profiles/${TAG}_shard1.25M_b64_* gpurun_out/profiles_new/
timeout -k 10 600 python -u bench.py > gpurun_out/bench_${TAG}_10M.json 2> gpurun_out/bench_${TAG}_10M.err
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 300 --warmup 10 --no-cpu > gpurun_out/bench_${TAG}_shard1.25M.json 2>&1
