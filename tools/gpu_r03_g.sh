# round 3: row-part knobs at 10M, k = 100 and 45 (refresh period, early refresh)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
ROWS=10000000 STEPS=100 EXTRA="--k 100" timeout -k 10 900 bash tools/ab_env.sh "" "HIPRAG_REFRESH=8" "HIPRAG_REFRESH=2" "HIPRAG_EARLY_REFRESH=1" > $O/ab_k100.log 2>&1
echo "ab k100 rc=$?"; cat $O/ab_k100.log
ROWS=10000000 STEPS=100 EXTRA="--k 45" timeout -k 10 900 bash tools/ab_env.sh "" "HIPRAG_REFRESH=8" "HIPRAG_EARLY_REFRESH=1" > $O/ab_k45.log 2>&1
echo "ab k45 rc=$?"; cat $O/ab_k45.log
