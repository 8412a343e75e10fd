#!/bin/bash
# Build an alternative libldpc_mi355x.so with one kernel source compiled with
# extra defines, for kernel experiments on the GPU box (LDPC_MI355X_LIB=...):
#   tools/build_variant.sh <name> [<src>.hip] -DLDPC_C3_MSLEEP=0 ...
#     -> var/variants/<name>/libldpc_mi355x.so   (<src> default coop3.hip; var/ travels to the GPU box)
# coop3.hip stands for the whole coop3 decoder: its host side and the six
# per-degree kernel objects (coop3_deg.hip -DC3_DEG=...), compiled in parallel.
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
skip="/$base.o\$"
vobjs="$out/$base.o"
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c -o "$out/$base.o" ldpcgputegra_amd/csrc/$src &
if [ "$src" = coop3.hip ]; then
    skip="/coop3(_d[0-9]+)?\.o\$"
    for d in 7 10 14 22 27 30; do
        /opt/rocm/bin/hipcc $HIPFLAGS "$@" -DC3_DEG=$d -c -o "$out/coop3_d$d.o" ldpcgputegra_amd/csrc/coop3_deg.hip &
        vobjs="$vobjs $out/coop3_d$d.o"
    done
fi
wait
objs=$(ls build/obj/*.o | grep -Ev "$skip")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libldpc_mi355x.so" $objs $vobjs
rm -f $vobjs
# the variant's extra defines, folded into _lib.source_hash() (bench.py keys PMC traffic by it)
echo "$src $*" > "$out/libldpc_mi355x.so.defines"
echo "$out/libldpc_mi355x.so"
