# Staged chunking variants: bottom-up dealing (DG_STAGED_SUB_FIRST), piece size (DG_STAGED_PIECE)
set -o pipefail
bash scripts/simP_ab.sh r6ab 8 base DG_STAGED_SUB_FIRST=1 DG_STAGED_PIECE=0.7 DG_STAGED_PIECE=1.0 base DG_STAGED_SUB_FIRST=1 || exit $?
REPS=2 bash scripts/ab.sh r6abP "--config P --steps 50 --warmup 5" DG_STAGED_SUB_FIRST=1 || exit $?
