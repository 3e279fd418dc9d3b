# One GPU call for front-end work: the front-end GPU tests, the bench's front-end section on a small
# eval batch, and a rocprofv3 kernel trace of cold 1 024-state calls (profiles/fe_trace.py).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_front.py tests/test_gpu_determinism.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fe1_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/fe1_tests.log; exit 1; }
tail -2 gpurun_out/fe1_tests.log
timeout -k 10 300 python -u bench.py --states 65536 --steps 2 --warmup 1 --keccak 0 --no-cpu --refute-sample 0 --suite 0 --suite-open-sweep 0 --div-split 0 --guided-sample 0 > gpurun_out/fe1_bench.json 2> gpurun_out/fe1_bench.err || { echo "bench failed"; tail -20 gpurun_out/fe1_bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fe_trace -o run --output-format csv -- python3 profiles/fe_trace.py > gpurun_out/fe1_trace.log 2> gpurun_out/fe1_trace.err || { echo "trace failed"; tail -20 gpurun_out/fe1_trace.err; exit 1; }
cat gpurun_out/fe1_trace.log
