set -e
bash profiles/run_cpw.sh d > gpurun_out/cpw_d.log 2>&1
