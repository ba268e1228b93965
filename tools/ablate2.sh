# Small-shard ablation: candidate appends, refresh, sample size (timing experiments only)
set -u
run() { echo "== $*"; env "$@" timeout -k 10 200 python tools/sweep.py 1.25e6 1e7 || exit 1; }
run HIPRAG_X=0
run HIPRAG_SCAN_DEBUG=1
run HIPRAG_SCAN_DEBUG=2
run HIPRAG_SAMPLE_DIV=16
run HIPRAG_SAMPLE_DIV=16 HIPRAG_SAMPLE_MIN=2048
run HIPRAG_SAMPLE_MIN=2048
run HIPRAG_REFRESH=2
run HIPRAG_RING=8
