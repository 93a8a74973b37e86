set -o pipefail
export TMPDIR=/tmp
for a in 0 8 1 2 4 3 5 6 7; do
  echo "== abl $a" >> gpurun_out/xs_abl.log
  MMT_XS_ABL=$a timeout -k 10 120 python tools/xs_bench.py >> gpurun_out/xs_abl.log 2>&1 || exit 1
done
