# Gather launches' groups smallest first (DG_SMALL_FIRST): config P N = 8 / 4 rank shares, one GPU
set -o pipefail
bash scripts/simP_ab.sh r6x 8 base DG_SMALL_FIRST=1 base DG_SMALL_FIRST=1 || exit $?
bash scripts/simP_ab.sh r6x4 4 base DG_SMALL_FIRST=1 || exit $?
bash scripts/sim_ab.sh r6xs 8 rccl:base rccl:DG_SMALL_FIRST=1 || exit $?
REPS=1 bash scripts/ab.sh r6xP "--config P --steps 50 --warmup 5" DG_SMALL_FIRST=1 || exit $?
