# SQ counters of single conv / wgrad launches (kbench specs in PMC_SPECS), one rocprofv3
# --pmc pass per counter group (<= 8 SQ counters per pass); GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); export TMPDIR=/tmp
SPECS="${PMC_SPECS:-c:256:64:64:6 c:128:128:128:6 c:64:256:256:6}"
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
G2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
G3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
i=0
for g in "$G1" "$G2" $( [ -n "$PMC_TCC" ] && echo "G3" ); do
  [ "$g" = "G3" ] && g="$G3"
  i=$((i+1))
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv \
      -d "$ROOT/gpurun_out/pmchr$i" -o run -- python "$ROOT/tools/kbench.py" --iters 3 $SPECS ) \
      > gpurun_out/pmchr$i.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"; tail -n 2 gpurun_out/pmchr$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python tools/pmc_show.py gpurun_out/pmchr1 gpurun_out/pmchr2 $( [ -n "$PMC_TCC" ] && echo gpurun_out/pmchr3 ) > gpurun_out/pmchr.txt 2>&1
echo pmc done
