#!/bin/bash
# Host-path leg under environment variants (development tool):
#   dev/scripts/host_env.sh OUT "ENV1 ENV2 ..."   (ENV: VAR=val,VAR2=val or "base")
set -o pipefail
o=gpurun_out/$1; mkdir -p $o
for E in $2; do
  EV=""; [ "$E" != base ] && EV=$(echo $E | tr ',' ' ')
  for i in 1 2; do
    env $EV timeout -k 10 150 python -u dev/scripts/host_probe.py > $o/h.tmp 2>&1 || { tail -5 $o/h.tmp; exit 1; }
    echo "$E $(grep '^{' $o/h.tmp)" | tee -a $o/host.txt
  done
done
