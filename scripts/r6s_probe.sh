# Config P rank shares with staged row pieces: the drug-target relation's LPT cost sweep
set -o pipefail
bash scripts/simP_ab.sh r6s 8 base DG_SHARD_GROUP_TAIL=150000 DG_SHARD_GROUP_TAIL=220000 DG_SHARD_GROUP_TAIL=300000 || exit $?
bash scripts/simP_ab.sh r6s4 4 DG_SHARD_GROUP_TAIL=220000 || exit $?
