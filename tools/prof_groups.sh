export TMPDIR=/tmp
for B in 128 64; do
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_scan -T -d gpurun_out/p${B}f -o run --output-format csv -- python3 bench.py --batch $B --steps 10 --warmup 2 --no-cpu > gpurun_out/p${B}f.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_scan -T -d gpurun_out/p${B}h -o run --output-format csv -- python3 bench.py --batch $B --steps 10 --warmup 2 --no-cpu > gpurun_out/p${B}h.log 2>&1 || exit 1
done
