# A/B of scan knobs on one box (timing experiments only): alternating runs
set -u
for rep in 1 2; do
  for wm in 0 1; do echo "== WAVE_MAJOR=$wm rep=$rep"; HIPRAG_WAVE_MAJOR=$wm timeout -k 10 200 python tools/sweep.py 1.25e6 1e7 || exit 1; done
done
