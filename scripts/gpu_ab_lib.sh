# A/B of the eval step across library builds (bench.py steps only):
#   bash scripts/gpu_ab_lib.sh tag=path/to/libmgp.so ...   ("base" = the in-tree library)
mkdir -p gpurun_out
run() {
  tag=$1; lib=$2
  MGP_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --steps 6 --warmup 2 --frontend 0 --suite 0 --suite-open-sweep 0 --keccak 0 --no-cpu --div-split 0 --refute-sample 0 --guided-sample 0 > gpurun_out/ablib_$tag.json 2> gpurun_out/ablib_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/ablib_$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ablib_$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step'], 3), round(d['roofline']['frac'], 4))"
}
for spec in "$@"; do
  tag=${spec%%=*}; lib=${spec#*=}
  [ "$lib" = "base" ] && lib=""
  run "$tag" "$lib" || exit 1
done
