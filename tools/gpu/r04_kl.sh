# r04 k+l in one call: the stagger A/B (r04_l.sh), then the whole GPU suite (r04_k.sh)
set -u
bash tools/gpu/r04_l.sh || exit $?
bash tools/gpu/r04_k.sh
