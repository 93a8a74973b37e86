#!/bin/bash
# round-end checks: GPU suite + smoke, then the 2-rank gloo rehearsal of the N > 1 bench path
set -o pipefail
bash tools/gpu_all.sh && bash tools/gpu_ddp_rehearsal.sh
