# rocprofv3 passes over the headline bench (kernel trace + stats, then HBM PMC counters).
# Usage on the GPU box: bash tools/profile.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
ARGS=${@:-"--steps 10 --warmup 2 --no-cpu"}
# the PMC passes only need the kernels: skip the CPU legs there (the kernel-trace pass runs ARGS as given)
PARGS="$ARGS"
case " $PARGS " in *" --no-cpu "*) ;; *) PARGS="$PARGS --no-cpu" ;; esac
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/kt -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_kt.log 2>&1
rc=$?; echo "kernel-trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_scan|k_filter' -T -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py $PARGS > $OUT/bench_pmc1.log 2>&1
rc=$?; echo "pmc FETCH_SIZE rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_scan|k_filter' -T -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py $PARGS > $OUT/bench_pmc2.log 2>&1
rc=$?; echo "pmc WRITE_SIZE rc=$rc"; [ $rc -ne 0 ] && exit $rc
# MFMA pipe: SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over SIMDs) against GRBM_GUI_ACTIVE (summed over 8 XCDs)
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex 'k_scan|k_filter' -T -d $OUT/pmc_mfma -o run --output-format csv -- python3 bench.py $PARGS > $OUT/bench_pmc3.log 2>&1
echo "pmc MFMA rc=$?"
find $OUT -name "*.csv"
