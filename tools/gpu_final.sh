#!/bin/bash
# end-of-round: measurement (PMC passes, bench line, profiles) then the GPU suite + smoke
set -o pipefail
bash tools/gpu_measure.sh ${1:-r02_b512} && bash tools/gpu_all.sh
