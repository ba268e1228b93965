# A/B: threshold refresh cadence (a refresh drains the corpus ring: vmcnt(0)) at 1.25M and 10M rows
set -e
for v in "HIPRAG_REFRESH=4" "HIPRAG_REFRESH=8" "HIPRAG_REFRESH=16" "HIPRAG_SCAN_DEBUG=2"; do
  env $v timeout -k 10 120 python -u bench.py --rows 1250000 --steps 300 --warmup 10 --no-cpu > gpurun_out/abr_1.25M_$(echo $v | tr '=' '_').json 2>/dev/null
  env $v timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/abr_10M_$(echo $v | tr '=' '_').json 2>/dev/null
done
