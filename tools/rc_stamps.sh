bash tools/round_check.sh || exit 1
CFGS="512,3" bash tools/stamps.sh
