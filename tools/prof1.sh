set -o pipefail
export TMPDIR=/tmp
cd /root/repo
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof1.log 2>&1
echo "exit $?" >> gpurun_out/prof1.log
find gpurun_out/prof1 -name "*stats*" | head >> gpurun_out/prof1.log
