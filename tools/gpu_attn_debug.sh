#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/attn_debug.py > gpurun_out/attn_debug.log 2>&1
