set -o pipefail
mkdir -p gpurun_out/tprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tprof -o run -- python3 $GRAFT_REPO_ROOT/tools/tome_bench.py > $GRAFT_REPO_ROOT/gpurun_out/tome_bench.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
find gpurun_out/tprof -name "*kernel_stats.csv" | head -3
exit $rc
