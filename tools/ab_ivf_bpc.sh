# A/B: IVF list-scan grid (blocks of 4 waves per CU)
set -e
for v in 8 3 2 4 16; do
  HIPRAG_IVF_BPC=$v timeout -k 10 300 python3 tools/bench_ivf.py --dist isotropic --steps 20 > gpurun_out/abivf_bpc$v.jsonl 2>/dev/null
done
