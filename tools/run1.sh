set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/r1_tests.log 2>&1; echo "tests exit $?" >> gpurun_out/r1_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r1_bench.log 2>&1; echo "bench exit $?" >> gpurun_out/r1_bench.log
