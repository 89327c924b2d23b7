# Run one gpurun call, retrying ONLY while no box could be acquired (no free slot / infrastructure back-off /
# a box that stopped responding while being prepared: nothing of the command ran, nothing was charged).  A
# call whose command ran is never repeated.  usage: bash scripts/gpurun_acquire.sh <log> <timeout> '<command>'
log=$1; lim=$2; cmd=$3
for attempt in $(seq 1 20); do
  timeout $((lim + 1500)) /usr/local/graft/bin/gpurun --timeout $lim -- "$cmd" > $log 2>&1
  if grep -q "no free box\|backing off\|stopped responding while being prepared\|slot(s) on this pod are busy\|retry in a few minutes\|taken away by the GPU service" $log && ! grep -q "status=ok\|status=fail\|EXIT" $log; then
    sleep 120
    continue
  fi
  break
done
echo "done (attempt $attempt)" >> $log
