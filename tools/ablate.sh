timeout -k 10 600 python -m pytest tests/ -q -m gpu --timeout 300 -x > gpurun_out/t_abl.log 2>&1; rc=$?; tail -3 gpurun_out/t_abl.log; [ $rc -ne 0 ] && exit $rc
for p in 16 8; do for r in 2 4 8; do echo "RING=$p REFRESH=$r"; HIPRAG_RING=$p HIPRAG_REFRESH=$r timeout -k 10 200 python tools/sweep.py 1.25e6 2.5e6 1e7 || exit 1; done; done
