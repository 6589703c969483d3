#!/bin/bash
# A/B: "<label>|<env>|<libdir>" specs, 2 interleaved rounds
for r in 1 2; do for spec in "$@"; do
  IFS='|' read -r label envs lib <<< "$spec"
  env $envs timeout -k 5 120 python ${RUNPY:-tools/diag/run.py} $lib ${MATRIX:-cant} | sed "s|^|$label |" || exit $?
done; done
