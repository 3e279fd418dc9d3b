mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4e_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r4e_tests.log; exit 1; }
tail -3 gpurun_out/r4e_tests.log
MGP_LIB_PATH=mutants/d/libmgp.so timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k mul_after_shift --timeout 60 --timeout-method thread > gpurun_out/r4e_mutd.log 2>&1; rc=$?; echo "mutant d rc=$rc" >> gpurun_out/r4e_mutd.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "mutant step abnormal rc=$rc"; exit 1; fi
tail -4 gpurun_out/r4e_mutd.log
timeout -k 10 60 ./profiles/issue_probe > gpurun_out/r4e_issue.json 2>&1 || { echo "probe failed"; exit 1; }
cat gpurun_out/r4e_issue.json
timeout -k 10 400 python -u bench.py > gpurun_out/r4e_bench.json 2> gpurun_out/r4e_bench.err || { echo "bench failed"; tail -20 gpurun_out/r4e_bench.err; exit 1; }
tail -c 600 gpurun_out/r4e_bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4e -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --frontend 0 --suite 0 --no-cpu --refute-sample 0 --guided-sample 0 > gpurun_out/r4e_prof_bench.json 2> gpurun_out/r4e_prof_bench.err || { echo "rocprof run failed"; tail -5 gpurun_out/r4e_prof_bench.err; exit 1; }
find gpurun_out/prof_r4e -name "*stats*" | head
