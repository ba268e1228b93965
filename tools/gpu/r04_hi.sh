# r04 h+i in one call: DPP refresh A/B + scan parity tests (r04_i.sh), then the embed probe (r04_h.sh)
set -u
bash tools/gpu/r04_i.sh || exit $?
bash tools/gpu/r04_h.sh
