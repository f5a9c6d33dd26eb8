#!/bin/bash
# GPU side of an A/B: abcheck.py with the default library and every build_variants/<v> named.
# usage: scripts/dev/ab_run.sh "<abcheck args>" v1 v2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
ARGS=$1; shift
timeout -k 10 120 python3 $R/scripts/dev/abcheck.py $ARGS || exit $?
for v in "$@"; do
  DSORT_LIB=$R/build_variants/$v/libdsort.so timeout -k 10 120 python3 $R/scripts/dev/abcheck.py $ARGS || exit $?
done
