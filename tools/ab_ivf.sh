# A/B: IVF scan ring depth (timing experiment only), 6.25M-row shard
set -u
for ring in 16 8 4; do
  echo "== ring=$ring"; HIPRAG_IVF_RING=$ring timeout -k 10 400 python -u tools/bench_rerank.py --steps 5 --no-exact --rerank-queries 1 || exit 1
done
