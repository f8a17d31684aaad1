#!/bin/bash
# Run a command on the GPU box via gpurun; re-submit only when the box could not be prepared
# (status=transient: nothing ran, nothing charged).  Usage: tools/gpu.sh <timeout> <command...>
T=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@" > gpurun_out/.gpu_call.log 2>&1
  rc=$?
  if grep -q "status=transient\|no box\|slot" gpurun_out/.gpu_call.log && ! grep -q "status=ok\|status=fail" gpurun_out/.gpu_call.log; then
    sleep 90; continue
  fi
  break
done
tail -3 gpurun_out/.gpu_call.log
exit $rc
