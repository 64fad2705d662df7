cd $GRAFT_REPO_ROOT
export PMC_COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES"
for sp in c:1024:16:32:6 c:1024:16:16:6 c:1024:32:16:521; do
  n=$(echo $sp | tr ':' '_')
  PMC_SPEC=$sp bash tools/gpu_check.sh pmcq > /dev/null && mv gpurun_out/pmcq gpurun_out/pmcA_$n || exit 1
  PMC_COUNTERS="FETCH_SIZE" PMC_SPEC=$sp bash tools/gpu_check.sh pmcq > /dev/null && mv gpurun_out/pmcq gpurun_out/pmcF_$n || exit 1
  PMC_COUNTERS="WRITE_SIZE" PMC_SPEC=$sp bash tools/gpu_check.sh pmcq > /dev/null && mv gpurun_out/pmcq gpurun_out/pmcW_$n || exit 1
done
