#!/bin/bash
# SQ counter passes (<= 8 SQ counters each, one pass per run) over kbench specs:
#   PMC_SPECS="w:128:128:256:0 c:128:128:128:6" bash tools/pmc_deep.sh
# Output: gpurun_out/pmcd_<n>/ per pass, summary by tools/pmc_show_deep.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROOT=$(pwd); export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM"
P3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES"
n=0
for P in "$P1" "$P2" "$P3"; do
  n=$((n+1))
  for c in $P; do grep -q "\b$c\b" gpurun_out/counters.txt || { echo "counter $c not listed: skipping pass $n"; continue 2; }; done
  ( cd /tmp && timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d "$ROOT/gpurun_out/pmcd_$n" -o run \
      -- python "$ROOT/tools/kbench.py" --iters 2 $PMC_SPECS ) > gpurun_out/pmcd_$n.log 2>&1
  rc=$?; echo "pass $n rc=$rc"; if [ $rc -ne 0 ]; then tail -n 5 gpurun_out/pmcd_$n.log; exit $rc; fi
done
echo pmc_deep done
