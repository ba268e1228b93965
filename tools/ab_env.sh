# 1.25M-row shard bench under several HIPRAG_* settings, two alternating repeats.
# Usage: [ROWS=n STEPS=n EXTRA='--k 100'] bash tools/ab_env.sh "ENV=.." "ENV=.." ...   ("" = defaults); prints step ms, FILTER ms, SAMPLE ms
mkdir -p gpurun_out
ROWS=${ROWS:-1250000}
STEPS=${STEPS:-300}
EXTRA=${EXTRA:-}
for rep in 1 2; do
  i=0
  for envs in "$@"; do
    i=$((i+1))
    env $envs timeout -k 10 120 python -u bench.py --rows $ROWS --steps $STEPS --warmup 10 --no-cpu $EXTRA > gpurun_out/abe_${i}_$rep.json 2>/dev/null || { echo "[$i] ${envs:-defaults} failed rc=$?"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abe_${i}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('[$i] rep $rep ${envs:-defaults}:', d['ms_per_step'], r['avg_launch_ms'], r['sample_pass_ms'])"
  done
done
