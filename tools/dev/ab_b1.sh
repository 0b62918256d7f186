#!/bin/bash
# dev: A/B of the single-slot stages between two library variants (Q3T_DEV_LIB names), alternating, 3 rounds
A=$1; B=$2
for r in 1 2 3; do for v in $A $B; do
  for st in 0 1; do printf "%s stage %s: " $v $st; Q3T_DEV_LIB=$v timeout -k 10 120 python3 tools/dev/stage_only.py $st 1 266 200 || exit 1; done
done; done
