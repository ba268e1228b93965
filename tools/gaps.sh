# Kernel-trace timelines of the 1.25M-row shard bench under several HIPRAG_* settings.
# Usage on the GPU box: bash tools/gaps.sh "ENV=.. ENV2=.." "ENV=.." ...   ("" = defaults)
export TMPDIR=/tmp
i=0
for envs in "$@"; do
  i=$((i+1)); d=gpurun_out/gaps_$i; mkdir -p $d
  echo "=== [$i] ${envs:-defaults}"
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 bench.py --rows ${ROWS:-1250000} --steps 20 --warmup 3 --no-cpu > $d/bench.log 2>&1 || { echo "rc=$?"; tail -3 $d/bench.log; exit 1; }
  python tools/timeline.py $(find $d -name "*kernel_trace.csv" | head -1) ${STEPS_SHOWN:-0}
done
