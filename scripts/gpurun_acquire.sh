# Run one gpurun call, retrying ONLY while no box could be acquired or the box was lost to the GPU service
# (gpurun status "transient": nothing charged, not a strike, its outputs are not pulled back).  A call whose
# command ran to a verdict of its own is never repeated.
# usage: bash scripts/gpurun_acquire.sh <log> <timeout> '<command>'
log=$1; lim=$2; cmd=$3
for attempt in $(seq 1 20); do
  timeout $((lim + 1500)) /usr/local/graft/bin/gpurun --timeout $lim -- "$cmd" > $log 2>&1
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status', ''))" 2>/dev/null)
  if grep -q "status=transient\|no free box\|backing off\|stopped responding while being prepared\|slot(s) on this pod are busy\|retry in a few minutes\|taken away by the GPU service" $log && { [ "$st" = "transient" ] || ! grep -q "status=ok\|status=fail" $log; }; then
    sleep 90
    continue
  fi
  break
done
echo "done (attempt $attempt)" >> $log
