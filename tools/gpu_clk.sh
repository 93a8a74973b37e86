#!/bin/bash
mkdir -p gpurun_out
out=gpurun_out/ntclk.log; : > $out
# warm the clock up first (several seconds of the same launch) then trace
for b in nt_trace nt_trace_NO_LOAD nt_trace_NO_MFMA; do
  for a in "70656 1536 384 5" "4096 4096 4096 5"; do
    echo "== $b $a" >> $out
    timeout -k 5 60 ./tools/$b $a 2>&1 | grep -E "^M=|clock" >> $out || exit 1
  done
done
