set -o pipefail
export TMPDIR=/tmp
for e in "X=0" "ROC_SIGNAL_POOL_SIZE=4096" "ROC_AQL_QUEUE_SIZE=65536" "DEBUG_CLR_MAX_BATCH_SIZE=4096" "AMD_DIRECT_DISPATCH=0" "ROC_ACTIVE_WAIT_TIMEOUT=0" "ROC_ACTIVE_WAIT_TIMEOUT=500" "HIP_FORCE_DEV_KERNARG=1" "X=1"; do
  out=$(env $e timeout -k 10 120 python tools/host_enqueue.py --steps 40) || { echo "$e failed"; exit 1; }
  echo "$e $out"
done
