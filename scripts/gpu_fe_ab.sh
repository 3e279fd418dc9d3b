# A/B of the front end's candidate-generation kernel choice (MGP_FE_ROWBLOCK=0/1) on cold
# 1 024-state calls, under a kernel trace: bash scripts/gpu_fe_ab.sh <tag>
set -e
tag=${1:-ab}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rb in 0 1; do
  MGP_FE_ROWBLOCK=$rb FE_REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fe_${tag}_rb$rb -o run --output-format csv -- python3 profiles/fe_trace.py > gpurun_out/fe_${tag}_rb$rb.log 2> gpurun_out/fe_${tag}_rb$rb.err || { echo "rb=$rb failed"; tail -20 gpurun_out/fe_${tag}_rb$rb.err; exit 1; }
  echo "rb=$rb"; cat gpurun_out/fe_${tag}_rb$rb.log
done
