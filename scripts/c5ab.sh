# Config-5 variant check + A/B: each variant's config-5 GPU tests, then the D bench beside the
# default library (scripts/ab.sh).  Usage: bash scripts/c5ab.sh TAG VARIANT...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
for v in "$@"; do
  DG_LIB=$PWD/decagon_amd/lib/var_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_config5.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$tag/test_$v.log 2>&1; rc=$?
  echo "$v tests rc=$rc: $(tail -1 gpurun_out/$tag/test_$v.log)"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
REPS=${REPS:-2} bash scripts/ab.sh $tag "--config D --steps 100 --warmup 10 --no-cpu-baseline" "$@"
