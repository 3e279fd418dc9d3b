set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
bash profiles/run_ab.sh xs2
timeout -k 10 200 python -u profiles/uop_costs.py --engine asm > gpurun_out/uopcost_xs2.txt 2>&1
grep "SIMD-cycles" gpurun_out/uopcost_xs2.txt
