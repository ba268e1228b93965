# r04 h: where the query embed's time goes (host tokenise / dispatch vs GPU), and a HIP-graph replay of it
set -u
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 300 python3 tools/embed_probe.py > $O/embed_probe.json 2> $O/embed_probe.err; rc=$?
echo "probe rc=$rc"; cat $O/embed_probe.json; [ $rc -ne 0 ] && tail -20 $O/embed_probe.err
exit $rc
