# Targeted GPU check: the given pytest node ids / -k expression, then (optional) one bench run.
# Usage (from gpurun): bash scripts/gpu_quick.sh <tag> "<pytest args>" [bench]
tag=$1; targs=$2; bench=${3:-}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest $targs -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_tests.log
if [ -n "$bench" ]; then
  timeout -k 10 400 python -u bench.py --detail gpurun_out/${tag}_bench_detail.json > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
  tail -c 1500 gpurun_out/${tag}_bench.json
fi
