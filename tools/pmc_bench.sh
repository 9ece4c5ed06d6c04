#!/bin/bash
# rocprofv3 PMC passes (SQ issue / wait counters, LDS array and HBM bytes)
# over bench.py's own workload, one pass per counter group, each under its
# own time limit; the CSVs are reduced in place by pmc_reduce.py.
# usage (on the GPU box): tools/pmc_bench.sh <outdir> <config> [op]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1; cfg=$2; op=${3:-protect}
export TMPDIR=/tmp
mkdir -p "$out"
passes=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  d="$out/p$i"
  echo "[pmc] $cfg pass $i: $p"
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $p --output-format csv -d "$d" -o p \
      -- python3 bench.py --config $cfg --op $op --steps 2 --warmup 1 \
         --no-cpu-baseline --traffic off > "$d.log" 2>&1
  rc=$?
  echo "[pmc] pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$d.log"; exit $rc; fi
  python3 tools/pmc_reduce.py "$d" || exit 1
done
