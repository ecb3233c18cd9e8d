set -o pipefail
bash scripts/simP_ab.sh r6n_p8 8 base DG_STAGED_BLOCKS=512 DG_STAGED_BLOCKS=128 DG_STAGED_BINS=256 || exit $?
