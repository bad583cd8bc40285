#!/bin/bash
# run several GPU step scripts in order; stop at the first that times out, aborts or faults
for s in "$@"; do
  bash "$s"
  rc=$?
  echo "== $s rc=$rc"
  case $rc in 124|137|134|139|143) echo "stopping after $s"; exit $rc;; esac
done
