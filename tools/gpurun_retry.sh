#!/bin/bash
# Re-submit a gpurun call only when no box was obtained (exit 3: nothing ran,
# nothing charged).  Any other outcome -- including a failing GPU command --
# is returned as is; the command itself is never retried.
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 60
done
exit 3
