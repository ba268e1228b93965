# round 3: the 8-rank bench flow rehearsed on one GPU (gloo, every rank on GPU 0, HIPRAG_BENCH_REHEARSE=1): the
# launcher, 8 shards of the 10M corpus, the 8-way packed all-gather + merge, recall vs the oracle.  Never the
# measured configuration (8 ranks share one GPU's HBM and the exchange takes the host path)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HIPRAG_BENCH_REHEARSE=1
O=gpurun_out/r03reh
mkdir -p $O
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 5 --recall-queries 4 > $O/rehearse8.json 2> $O/rehearse8.err
rc=$?; echo "rehearse 8 rc=$rc"; tail -c 1500 $O/rehearse8.json; tail -5 $O/rehearse8.err
exit $rc
