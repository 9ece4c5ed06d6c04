#!/bin/bash
# round-4 GPU session 8: k_gcm LDS budget -- the AES tables read with 16 of
# their 32 copies (what conflict-free GHASH tables would have to pay for
# room: two copies of the per-position tables need 32 KiB more than LDS
# has), timing and SQ_LDS_BANK_CONFLICT against the tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="gcm_rep16" tools/step_variants.sh gcm256 2 || exit 1
for v in tree gcm_rep16; do
  lib=$PWD/libsrtp_amd/libsrtp_mi355x.so
  [ $v = tree ] || lib=$PWD/exp_build/$v/libsrtp_mi355x.so
  LIBSRTP_MI355X_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES \
      --output-format csv -d gpurun_out/s8_pmc_$v -o p -- python3 bench.py --config gcm256 --steps 2 --warmup 1 \
      --no-cpu-baseline --traffic off > gpurun_out/s8_pmc_$v.log 2>&1 || { tail -5 gpurun_out/s8_pmc_$v.log; exit 1; }
  python3 tools/pmc_reduce.py gpurun_out/s8_pmc_$v
  echo "== $v"; grep -rh k_gcm gpurun_out/s8_pmc_$v --include=pmc_summary.csv || true
done
