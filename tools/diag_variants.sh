#!/bin/bash
# tools/diag_mpc.py under several environment settings; stops at a timeout / abort / crash
set -o pipefail
CASE=${1:-ex10}; SCALE=${2:-0.05}; shift 2
[ $# -eq 0 ] && set -- "-" "MADIPM_FOLD=0" "MADIPM_FACT_PIPE=0" "MADIPM_TREE_SOLVE=0"
for E in "$@"; do
  [ "$E" = "-" ] && E=""
  echo "== ${E:-default}"
  env $E timeout -k 10 120 python -u tools/diag_mpc.py $CASE $SCALE 2>&1 | tail -3
  rc=$?; case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
