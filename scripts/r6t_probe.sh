# Epilogue partial loads in flight (8 default; variants 4, 16) and the drug-target LPT cost sweep
set -o pipefail
bash scripts/simP_ab.sh r6t 8 base epib4 epib16 DG_SHARD_GROUP_TAIL=150000 DG_SHARD_GROUP_TAIL=250000 || exit $?
REPS=1 bash scripts/ab.sh r6tP "--config P --steps 50 --warmup 5" epib4 || exit $?
REPS=2 bash scripts/ab.sh r6tS "--steps 200 --warmup 20 --no-extra" epib4 || exit $?
