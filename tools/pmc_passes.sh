#!/bin/bash
# rocprofv3 PMC passes over the bench workload (one counter group per run:
# gfx950 slots are SQ 8, TCC 4 with FETCH_SIZE=3 / WRITE_SIZE=2).
# usage (on the GPU box): tools/pmc_passes.sh <outdir> [bench args...]
# Each pass runs under its own time limit; the script stops at the first
# pass that times out or faults.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=${1:-gpurun_out/pmc}; shift
args=${*:-"--steps 2 --warmup 1 --no-cpu-baseline"}
export TMPDIR=/tmp
mkdir -p "$out"
passes=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_64B_sum"
  "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum"
  "TA_BUSY_avr TA_BUSY_max"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  echo "[pmc] pass $i: $p"
  timeout -k 10 240 rocprofv3 --pmc $p --output-format csv -d "$out/p$i" -o p \
      -- python3 bench.py $args > "$out/p$i.log" 2>&1
  rc=$?
  echo "[pmc] pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/p$i.log"; exit $rc; fi
done
