# GPU box: memory-feed counters of single conv launches (kbench specs in PMC_SPECS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
SPECS="${PMC_SPECS:-c:128:128:128:6 c:32:512:512:0}"
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
G2="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES GRBM_GUI_ACTIVE"
G3="TCC_HIT TCC_MISS TCC_BUSY TA_DATA_STALLED_BY_TC_CYCLES TA_BUFFER_READ_LDS_WAVEFRONTS GRBM_GUI_ACTIVE"
i=0
for g in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  ( cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $g --output-format csv \
      -d "$ROOT/gpurun_out/pmcf$i" -o run -- python "$ROOT/tools/kbench.py" --iters 3 $SPECS ) \
      > gpurun_out/pmcf$i.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"; tail -n 2 gpurun_out/pmcf$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python tools/pmc_show.py gpurun_out/pmcf1 gpurun_out/pmcf2 gpurun_out/pmcf3 > gpurun_out/pmcf.txt 2>&1
echo pmc done
