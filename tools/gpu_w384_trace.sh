set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/wtr -o run --output-format csv -- python tools/w384_one.py 138496 384 1536 > gpurun_out/wtr.log 2>&1 &&
MMT_W384_MT=256 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/wtr2 -o run --output-format csv -- python tools/w384_one.py 131072 384 1536 > gpurun_out/wtr2.log 2>&1 &&
MMT_W384_MT=64 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/wtr3 -o run --output-format csv -- python tools/w384_one.py 7424 384 1536 > gpurun_out/wtr3.log 2>&1
