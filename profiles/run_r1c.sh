set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r1c_tests.log 2>&1
tail -3 gpurun_out/r1c_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r1c_bench.json 2> gpurun_out/r1c_bench.err
cat gpurun_out/r1c_bench.json
