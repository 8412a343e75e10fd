#!/bin/bash
# Build an alternative libldpc_mi355x.so whose coop2.hip is compiled with
# extra defines, for kernel experiments on the GPU box (LDPC_MI355X_LIB=...):
#   tools/build_variant.sh <name> -DLDPC_COOP2_R=4 ...   -> build/variants/<name>/libldpc_mi355x.so
# Run in the dev container after `make -C ldpcgputegra_amd/csrc` (reuses its objects).
set -e
cd "$(dirname "$0")/.."
name=$1
shift
out=build/variants/$name
mkdir -p "$out"
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function"
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c -o "$out/coop2.o" ldpcgputegra_amd/csrc/coop2.hip
objs=$(ls build/obj/*.o | grep -v '/coop2.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libldpc_mi355x.so" $objs "$out/coop2.o"
echo "$out/libldpc_mi355x.so"
