# A/B of the bucket stream assignment (MGP_BUCKET_LPT=0 round-robin / 1 LPT), interleaved.
ARGS="--steps 10 --warmup 2 --keccak 0 --no-cpu --refute-sample 0 --frontend 0 --suite 0 --suite-open-sweep 0 --div-split 0 --guided-sample 0 --detail gpurun_out/ab_detail.json"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in 0 1; do
    MGP_BUCKET_LPT=$v timeout -k 10 120 python bench.py $ARGS > gpurun_out/ab_lpt_${v}_${rep}.json 2> gpurun_out/ab_lpt_${v}_${rep}.err || { echo "run failed"; tail -5 gpurun_out/ab_lpt_${v}_${rep}.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_lpt_${v}_${rep}.json').read().strip().splitlines()[-1]); print('lpt=$v rep=$rep', round(d['ms_per_step'],3), round(d['roofline']['launch_ms'],3))"
  done
done
