#!/bin/bash
# Experiment builds (never the product library): build/exp/<name>/libafm.so from the unchanged
# product sources with extra compile flags on every translation unit (A/B of compile-time knobs
# such as -DAFM_TAIL_PRIO=3).  Load with AFM_LIB=<path>.
#   tools/build_flags_variant.sh <name> <hipcc flags...>
set -e
R=$(cd $(dirname $0)/.. && pwd)
P=$R/alpha-multi-factor-models_amd
name=$1; shift
out=$P/build/exp/$name; mkdir -p $out
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I$R/include -I$P/csrc"
objs=""
for f in $P/csrc/*.hip $P/csrc/*.cpp; do
  b=$(basename $f)
  /opt/rocm/bin/hipcc $FLAGS "$@" -c $f -o $out/$b.o &
  objs="$objs $out/$b.o"
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/libafm.so $objs
echo $out/libafm.so
