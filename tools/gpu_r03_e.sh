# round 3: 1.25M-shard knob sweep (tools/ab_env.sh: two alternating repeats per setting)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 900 bash tools/ab_env.sh "" "HIPRAG_TAIL_CUS=16" "HIPRAG_TAIL_CUS=48" "HIPRAG_DYN_PCT=5" "HIPRAG_DYN_PCT=20" "HIPRAG_DYN_CHUNK=4" > $O/ab_shard1.25M.log 2>&1
echo "ab rc=$?"; cat $O/ab_shard1.25M.log
