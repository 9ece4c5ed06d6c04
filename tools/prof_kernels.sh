#!/bin/bash
# Kernel-trace stats plus the SQ / GRBM counter passes that explain a kernel's
# VALU / LDS balance, over a short bench.py run (each pass its own process
# and time limit; gfx950 slots: SQ 8, GRBM 2 per pass).
# usage (on the GPU box): tools/prof_kernels.sh <outdir> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=${1:-gpurun_out/prof}; shift
args=${*:-"--steps 3 --warmup 1 --no-cpu-baseline --traffic off"}
export TMPDIR=/tmp
mkdir -p "$out"
echo "[prof] kernel trace"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o kt \
    -- python3 bench.py $args > "$out/kt.log" 2>&1 || { tail -5 "$out/kt.log"; exit 1; }
python3 tools/pmc_reduce.py "$out/kt"
passes=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  echo "[prof] pass $i: $p"
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d "$out/p$i" -o p \
      -- python3 bench.py $args > "$out/p$i.log" 2>&1
  rc=$?
  echo "[prof] pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/p$i.log"; exit $rc; fi
  python3 tools/pmc_reduce.py "$out/p$i"
done
