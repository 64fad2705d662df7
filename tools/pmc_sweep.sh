# PMC stall breakdown of single conv / wgrad launches (tools/kbench.py specs); GPU box only
export PMC_COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES"
for spec in ${PMC_SPECS:-c:256:128:64:8 w:128:128:256:0 c:1024:16:16:6 w:1024:16:32:0}; do
  PMC_SPEC=$spec bash tools/gpu_check.sh pmcq || exit 1
  rm -rf gpurun_out/pmcq_${spec//:/_}
  mv gpurun_out/pmcq gpurun_out/pmcq_${spec//:/_}
done
