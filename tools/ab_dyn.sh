# A/B: dynamic tail share / run length of the FILTER scan (timing experiment only)
set -u
for rep in 1 2; do
  for cfg in "0 2" "10 2" "20 2" "20 4" "30 2"; do
    set -- $cfg
    echo "== pct=$1 chunk=$2 rep=$rep"; HIPRAG_DYN_PCT=$1 HIPRAG_DYN_CHUNK=$2 timeout -k 10 200 python tools/sweep.py 1.25e6 1e7 || exit 1
  done
done
