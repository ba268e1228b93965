# IVF stage timing + a rocprofv3 kernel trace of it (clustered and isotropic 6.25M x 1024 f16 shards).
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/bench_ivf.py > gpurun_out/ivf_r02.jsonl 2> gpurun_out/ivf_r02.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_ivf -o run --output-format csv -- python3 tools/bench_ivf.py --dist isotropic --steps 5 > gpurun_out/ivf_prof_r02.log 2>&1
