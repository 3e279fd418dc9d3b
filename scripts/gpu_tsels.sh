# GPU check of select-chain work: the select-chain parity tests, the whole -m gpu suite, and the
# bench's front-end section on a small eval batch (front-end rate, WalletLibrary 2-state latency).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "select_chain or uf_byte or spilled" > gpurun_out/ts_tests.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/ts_tests.log; exit 1; }
tail -2 gpurun_out/ts_tests.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ts_all.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/ts_all.log; exit 1; }
tail -2 gpurun_out/ts_all.log
timeout -k 10 300 python -u bench.py --states 65536 --steps 2 --warmup 1 --keccak 0 --no-cpu --refute-sample 0 --suite 0 --suite-open-sweep 0 --div-split 0 --guided-sample 0 > gpurun_out/ts_bench.json 2> gpurun_out/ts_bench.err || { echo "bench failed"; tail -20 gpurun_out/ts_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ts_bench.json')); fe=d['frontend']
print('fe', round(fe['states_per_s']), fe['calls_seconds'], 'gpu', round(fe['stages_ms']['gpu_wait_ms'],2))
print('wallet2', [(r['ms_per_call'], r['gpu_wait_ms']) for r in fe['latency_2_by_contract']['wallet']])
print('lat1024', [(r['ms_per_call'], r['gpu_wait_ms']) for r in fe['latency'] if r['states']==1024])"
