#!/bin/bash
# retry gpurun while no box is available (rc 3, or a transient pool status); usage: gr.sh TIMEOUT 'cmd' LOG
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout $1 -- "$2" > $3 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $3; then echo "rc=$rc" >> $3; exit $rc; fi
  echo "try $i: rc=$rc" >> $3.tries
  sleep 120
done
echo "rc=3 (gave up)" >> $3
