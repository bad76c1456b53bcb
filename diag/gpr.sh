#!/bin/bash
# (host side, this container) run a gpurun command, retrying only while no GPU slot is free (exit 3: nothing ran)
# usage: gpr.sh OUTFILE TIMEOUT 'command' — retries only while gpurun reports "no slot free" (exit 3: nothing ran)
out=$1; to=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1; rc=$?
  echo "EXIT $rc (attempt $i)" >> $out
  [ $rc -ne 3 ] && exit $rc
  sleep 60
done
