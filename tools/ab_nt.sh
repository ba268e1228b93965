# A/B: non-temporal vs default-policy corpus loads (timing experiment only)
set -u
for rep in 1 2; do
  echo "== nt rep=$rep"; timeout -k 10 200 python tools/sweep.py 1.25e6 1e7 || exit 1
  echo "== default rep=$rep"; HIPRAG_LIB_OVERRIDE=youtu-rag_amd/hiprag/libhiprag_ab.so timeout -k 10 200 python tools/sweep.py 1.25e6 1e7 || exit 1
done
