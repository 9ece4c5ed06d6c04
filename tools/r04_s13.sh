#!/bin/bash
# round-4 GPU session 13: the round-4 bench lines (PMC traffic + CPU
# baseline), the N=2 line (two ranks on the one GPU over gloo, session
# replicated from rank 0), the headline's rocprofv3 kernel-trace summary,
# the end-to-end (PCIe-inclusive) rates
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/${OUTDIR:-s13}
export TMPDIR=/tmp
run() {   # name, args...
  local name=$1; shift
  timeout -k 10 500 python3 bench.py "$@" > gpurun_out/${OUTDIR:-s13}/$name.json 2> gpurun_out/${OUTDIR:-s13}/$name.err || { tail -5 gpurun_out/${OUTDIR:-s13}/$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${OUTDIR:-s13}/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; c=d['cpu_baseline'] or {}; print('$name', round(d['value']/1e6,1), 'Mpkt/s', round(d['ms_per_step'],4), 'ms', r['kernel'], round(r['kernel_ms'],4), 'frac', round(r['frac'],4), 'traffic', r['traffic'], 'cpu', c.get('value'))"
}
run icm128 --steps 20 --warmup 3 || exit 1
run gcm256 --config gcm256 --steps 20 --warmup 3 || exit 1
run g711 --config g711 --steps 10 --warmup 3 || exit 1
run icm128_unp --op unprotect --steps 20 --warmup 3 --cpu-seconds 3 || exit 1
run icm128_unp_reorder --op unprotect --reorder 0.01 --dup 0.001 --steps 20 --warmup 3 --cpu-seconds 3 || exit 1
run g711_unp --config g711 --op unprotect --steps 10 --warmup 3 --cpu-seconds 3 || exit 1
SRTP_BENCH_DEVICE=0 SRTP_DIST_BACKEND=gloo OMP_NUM_THREADS=1 run gcm256_n2 --config gcm256 --gpus 2 --steps 10 --warmup 2 --cpu-seconds 3 --traffic off || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${OUTDIR:-s13}/kt_icm128 -o kt \
    -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --traffic off > gpurun_out/${OUTDIR:-s13}/kt_icm128.log 2>&1 || { tail -5 gpurun_out/${OUTDIR:-s13}/kt_icm128.log; exit 1; }
python3 tools/pmc_reduce.py gpurun_out/${OUTDIR:-s13}/kt_icm128
for op in protect unprotect; do
  timeout -k 10 300 ./tools/e2e_bench $((1<<20)) 1400 5 16 $op > gpurun_out/${OUTDIR:-s13}/e2e_$op.json 2> gpurun_out/${OUTDIR:-s13}/e2e_$op.err || exit 1
  cat gpurun_out/${OUTDIR:-s13}/e2e_$op.json
done
