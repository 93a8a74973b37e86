#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/nttrace.log
: > $out
for b in ${NT_BINS:-nt_trace nt_trace_nostore}; do
  for args in ${NT_ARGS:-"70656 1536 384 5" "70656 1536 384 6" "74752 384 384 6" "70656 384 1536 7" "70656 384 1536 7 1" "4096 4096 4096 5"}; do
    echo "== $b $args" >> $out
    timeout -k 5 60 ./tools/$b $args >> $out 2>&1 || exit 1
  done
done
