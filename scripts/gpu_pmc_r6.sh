# Round-6 PMC evidence: the full collection (profiles/collect.sh) and the division-free
# twin's SQ counters (MGP_SYNTH_ABLATE=nodiv) for the SALU / VALU split.
set -e
bash profiles/collect.sh r6 > gpurun_out/collect_r6.log 2>&1 || { echo "collect failed"; tail -20 gpurun_out/collect_r6.log; exit 1; }
tail -2 gpurun_out/collect_r6.log
COUNTERS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" bash profiles/pmc_pass.sh full > gpurun_out/pmc_full.txt 2>&1 || { echo "pmc full failed"; cat gpurun_out/pmc_full.txt; exit 1; }
cat gpurun_out/pmc_full.txt
MGP_SYNTH_ABLATE=nodiv COUNTERS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" bash profiles/pmc_pass.sh nodiv > gpurun_out/pmc_nodiv.txt 2>&1 || { echo "pmc nodiv failed"; cat gpurun_out/pmc_nodiv.txt; exit 1; }
cat gpurun_out/pmc_nodiv.txt
