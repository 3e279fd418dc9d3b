mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r4b_tests.log; exit 1; }
tail -3 gpurun_out/r4b_tests.log
MGP_LIB_PATH=mutants/d/libmgp.so timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k mul_after_shift --timeout 60 --timeout-method thread > gpurun_out/r4b_mutd.log 2>&1; rc=$?; echo "mutant d rc=$rc" >> gpurun_out/r4b_mutd.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "mutant step abnormal rc=$rc"; exit 1; fi
tail -4 gpurun_out/r4b_mutd.log
timeout -k 10 400 python -u bench.py > gpurun_out/r4b_bench.json 2> gpurun_out/r4b_bench.err || { echo "bench failed"; tail -20 gpurun_out/r4b_bench.err; exit 1; }
tail -c 600 gpurun_out/r4b_bench.json
