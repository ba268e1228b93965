# A/B: tail-stream pipelining vs one stream (timing experiment only)
set -u
for rep in 1 2; do
  echo "== overlap rep=$rep"; timeout -k 10 200 python tools/sweep.py 1.25e6 2.5e6 1e7 || exit 1
  echo "== one-stream rep=$rep"; HIPRAG_OVERLAP=0 timeout -k 10 200 python tools/sweep.py 1.25e6 2.5e6 1e7 || exit 1
done
