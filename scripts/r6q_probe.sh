# Config P rank shares: the drug-target relation's LPT cost (DG_SHARD_GROUP_TAIL, nonzeros)
set -o pipefail
bash scripts/simP_ab.sh r6q 8 base DG_SHARD_GROUP_TAIL=300000 DG_SHARD_GROUP_TAIL=600000 DG_SHARD_GROUP_TAIL=900000 || exit $?
bash scripts/simP_ab.sh r6q4 4 base DG_SHARD_GROUP_TAIL=600000 || exit $?
