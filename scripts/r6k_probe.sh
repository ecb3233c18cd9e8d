set -o pipefail
bash scripts/sim_ab.sh r6k_s2 2 rccl:base rccl:DG_TAB_BALANCE=0 peer:base peer:DG_TAB_BALANCE=0 || exit $?
bash scripts/sim_ab.sh r6k_s4 4 rccl:base peer:base || exit $?
