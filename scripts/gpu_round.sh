# One GPU validation pass at the current tree: -m gpu suite, bench, rocprofv3 kernel stats.
# Usage (from gpurun): bash scripts/gpu_round.sh <tag>
tag=${1:-r4f}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_tests.log
timeout -k 10 400 python -u bench.py --detail gpurun_out/${tag}_bench_detail.json > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
tail -c 600 gpurun_out/${tag}_bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --frontend 0 --suite 0 --no-cpu --refute-sample 0 --guided-sample 0 > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof_bench.err || { echo "rocprof run failed"; tail -5 gpurun_out/${tag}_prof_bench.err; exit 1; }
find gpurun_out/prof_${tag} -name "*stats*" | head
