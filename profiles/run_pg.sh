set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
bash profiles/run_ab.sh mul2
timeout -k 10 200 python -u profiles/uop_costs.py --engine asm > gpurun_out/uopcost_mul2.txt 2>&1
grep "SIMD-cycles" gpurun_out/uopcost_mul2.txt
