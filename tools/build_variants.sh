#!/bin/bash
# Builds timing-experiment variants of libsrtp_mi355x.so into
# exp_build/<name>/: one kernel translation unit recompiled with extra flags
# (TU=srtp_icm_nr10_km0: the AES-128 ICM kernel of uniform-key batches,
# km1 per-lane keys; TU=srtp_gcm_nr14 for the GCM-256 kernel),
# every other object taken from libsrtp_amd/build.  Compiles run in parallel.
# usage: [TU=srtp_gcm_nr14] tools/build_variants.sh name "-DFLAG ..." [name "-D..."]...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -j8 -C "$ROOT/libsrtp_amd"
TU=${TU:-srtp_icm_nr10_km0}
case $TU in
  srtp_gcm_nr*) SRC=$ROOT/libsrtp_amd/csrc/srtp_gcm.hip; EXTRA="-DGCM_NR=${TU#srtp_gcm_nr}";;
  srtp_icm_nr*_km*) SRC=$ROOT/libsrtp_amd/csrc/srtp_icm.hip
      nk=${TU#srtp_icm_nr}; EXTRA="-DICM_NR=${nk%_km*} -DICM_KM=${nk#*_km}";;
  *) SRC=$ROOT/libsrtp_amd/csrc/$TU.hip; EXTRA="";;
esac
OTHERS=$(ls $ROOT/libsrtp_amd/build/*.o | grep -v "/$TU.o$")
pids=()
names=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  d=$ROOT/exp_build/$name; mkdir -p $d
  ( /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 $EXTRA $flags \
       -I$ROOT/include -I$ROOT/libsrtp_amd/csrc -c $SRC -o $d/k.o &&
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $d/libsrtp_mi355x.so \
       $d/k.o $OTHERS && echo "built $name" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
