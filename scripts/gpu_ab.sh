# A/B of the eval step under launch settings (bench.py steps only).
mkdir -p gpurun_out
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 6 --warmup 2 --frontend 0 --suite 0 --keccak 0 --no-cpu --div-split 0 --refute-sample 0 --guided-sample 0 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/ab_$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step'], 3), round(d['roofline']['frac'], 4))"
}
run base MGP_AB=0 && run streams0 MGP_BUCKET_STREAMS=0 && run cpw1 MGP_CHUNKS_PER_WAVE=1 && run cpw2 MGP_CHUNKS_PER_WAVE=2 && run base2 MGP_AB=0
