#!/bin/bash
# SQ instruction counts of the bench kernels for the tree and exp_build
# variants (one rocprofv3 --pmc pass each), on the GPU box:
#   tools/pmc_lib_variants.sh <outdir> "<bench args>" name...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:?outdir}; args=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
for name in tree "$@"; do
  so=$PWD/libsrtp_amd/libsrtp_mi355x.so
  [ "$name" != tree ] && so=$PWD/exp_build/$name/libsrtp_mi355x.so
  LIBSRTP_MI355X_LIB=$so timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU \
      SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES \
      --output-format csv -d "$out/$name" -o p -- python3 bench.py $args \
      --steps 2 --warmup 1 --no-cpu-baseline --traffic off \
      > "$out/$name.log" 2>&1 || { tail -5 "$out/$name.log"; exit 1; }
  python3 - "$out/$name" "$name" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "k_icm" in k or "k_gcm" in k:
        agg[k.split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(sys.argv[2], k, {c: round(sum(v) / len(v) / 1e6, 2) for c, v in sorted(d.items())})
PY
done
