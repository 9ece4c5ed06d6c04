#!/bin/bash
# Builds timing-experiment variants of libsrtp_mi355x.so into exp_build/<name>/
# usage: tools/build_variants.sh name "-DFLAG ..." [name "-D..."]...
set -e
make -s -C "$(cd "$(dirname "$0")/.." && pwd)/libsrtp_amd"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  d=$ROOT/exp_build/$name; mkdir -p $d
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 $flags \
     -I$ROOT/include -I$ROOT/libsrtp_amd/csrc -c $ROOT/libsrtp_amd/csrc/srtp_kernels.hip -o $d/k.o &
  gcc -O2 -fPIC -std=gnu11 -I$ROOT/include -I$ROOT/libsrtp_amd/csrc -c $ROOT/libsrtp_amd/csrc/srtp_host.c -o $d/h.o
  gcc -O2 -fPIC -std=gnu11 -I$ROOT/include -I$ROOT/libsrtp_amd/csrc -c $ROOT/libsrtp_amd/csrc/host_crypto.c -o $d/c.o
  wait
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $d/libsrtp_mi355x.so $d/k.o $d/h.o $d/c.o $ROOT/libsrtp_amd/build/srtp_prepass.o
  echo built $name
done
