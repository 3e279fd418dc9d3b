set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
A="--states 65536 --steps 2 --warmup 1 --no-cpu --refute-sample 0 --frontend 0"
for B in 0 2048 4096 8192 16384; do
  MGP_KECCAK_BLOCKS=$B timeout -k 10 200 python -u bench.py $A > gpurun_out/kab_$B.json 2> gpurun_out/kab_$B.err
  python3 -c "import json;d=json.load(open('gpurun_out/kab_$B.json'));print($B, d['keccak']['value'], d['keccak']['roofline']['launch_ms'])"
done
