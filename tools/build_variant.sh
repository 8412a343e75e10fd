#!/bin/bash
# Build an alternative libldpc_mi355x.so with one kernel source compiled with
# extra defines, for kernel experiments on the GPU box (LDPC_MI355X_LIB=...):
#   tools/build_variant.sh <name> [<src>.hip] -DLDPC_COOP2_R=4 ...
#     -> var/variants/<name>/libldpc_mi355x.so   (<src> default coop3.hip; var/ travels to the GPU box)
# Run in the dev container after `make -C ldpcgputegra_amd/csrc` (reuses its objects).
set -e
cd "$(dirname "$0")/.."
name=$1
shift
src=coop3.hip
if [[ "$1" == *.hip ]]; then
    src=$1
    shift
fi
base=${src%.hip}
out=var/variants/$name
mkdir -p "$out"
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function"
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c -o "$out/$base.o" ldpcgputegra_amd/csrc/$src
objs=$(ls build/obj/*.o | grep -v "/$base.o\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libldpc_mi355x.so" $objs "$out/$base.o"
echo "$out/libldpc_mi355x.so"
