#!/bin/bash
# Counter passes over a short bench run (one rocprofv3 pass per counter group,
# --kernel-trace only; no sys/runtime tracing, per the pool rules).
# Usage: profiles/run_pmc.sh <outdir> <bench args...>
set -o pipefail
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
groups=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_FLAT"
)
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/pass$i" -o pmc -- python3 bench.py "$@" --no-cpu-baseline > "$out/pass$i.log" 2>&1 || { echo "pass $i ($grp) failed rc=$?"; tail -5 "$out/pass$i.log"; }
done
