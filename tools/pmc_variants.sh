#!/bin/bash
# Two rocprofv3 PMC passes (SQ issue/occupancy counters + clock) over the
# protect kernel of each exp_build/<name> variant (tools/time_variants.py
# --one NAME, run in-process), reduced on the box by pmc_reduce.py.
# usage (on the GPU box): [CFG=gcm256] tools/pmc_variants.sh <outdir> name [name...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
passes=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE"
)
for name in "$@"; do
  i=0
  for p in "${passes[@]}"; do
    i=$((i+1))
    d="$out/$name/p$i"; mkdir -p "$out/$name"
    echo "[pmc] $name pass $i"
    timeout -k 10 180 rocprofv3 --kernel-trace --pmc $p --output-format csv -d "$d" -o p \
        -- python3 tools/time_variants.py --one $name ${CFG:-icm128} > "$d.log" 2>&1
    rc=$?
    echo "[pmc] $name pass $i rc=$rc $(tail -1 $d.log)"
    if [ $rc -ne 0 ]; then tail -5 "$d.log"; exit $rc; fi
    python3 tools/pmc_reduce.py "$d" || exit 1
  done
done
