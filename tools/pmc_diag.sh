# SQ counters of one kbench spec with and without the conv_hr timing diagnostics (PG_HR_DIAG)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); export TMPDIR=/tmp
SPEC="${PMC_SPEC:-c:128:128:128:6}"
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
G2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
for dg in 0 7; do
i=0
for g in "$G1" "$G2"; do
  i=$((i+1))
  ( cd /tmp && PG_HR_DIAG=$dg timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv \
      -d "$ROOT/gpurun_out/pmcd${dg}_$i" -o run -- python "$ROOT/tools/kbench.py" --iters 3 $SPEC ) \
      > gpurun_out/pmcd${dg}_$i.log 2>&1
  rc=$?; echo "diag $dg group $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 gpurun_out/pmcd${dg}_$i.log; exit $rc; fi
done
python tools/pmc_show.py gpurun_out/pmcd${dg}_1 gpurun_out/pmcd${dg}_2 > gpurun_out/pmcd$dg.txt 2>&1
done
echo pmc done
