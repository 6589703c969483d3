#!/bin/bash
# interleave variants over 2 rounds
for r in 1 2; do for v in "$@"; do timeout -k 5 120 python tools/diag/run.py tools/diag/v$v ${MATRIX:-cant} || exit $?; done; done
