# round-3 end: rocprof passes over the default bench (10M headline) and the 1.25M shard with the final code,
# summaries into profiles/ (copied back through gpurun_out/profiles_new/), then the default bench line
set -e
TAG=r03final
bash tools/profile.sh ${TAG}_10M
bash tools/profile.sh ${TAG}_shard1.25M --rows 1250000 --steps 20 --warmup 3 --no-cpu
python3 tools/summarize_profile.py gpurun_out/prof_${TAG}_10M ${TAG}_10Mx1024_b64 20480000000 > /dev/null
python3 tools/summarize_profile.py gpurun_out/prof_${TAG}_shard1.25M ${TAG}_shard1.25M_b64 2560000000 > /dev/null
mkdir -p gpurun_out/profiles_new
cp profiles/${TAG}_10Mx1024_b64_* profiles/${TAG}_shard1.25M_b64_* gpurun_out/profiles_new/
timeout -k 10 600 python -u bench.py > gpurun_out/bench_${TAG}_10M.json 2> gpurun_out/bench_${TAG}_10M.err
cat gpurun_out/bench_${TAG}_10M.json
