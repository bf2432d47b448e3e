#!/bin/bash
# Experiment builds (never the product library): build/exp/<name>/libafm.so from the product
# sources with one translation unit replaced by an edited copy.  Load with AFM_LIB=<path>.
#   tools/build_variant.sh <name> <edited.hip> [extra hipcc flags]
set -e
R=$(cd $(dirname $0)/.. && pwd)
P=$R/alpha-multi-factor-models_amd
name=$1; src=$2; shift 2
out=$P/build/exp/$name; mkdir -p $out
base=$(basename $src)
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I$R/include -I$P/csrc"
objs=""
for f in $P/csrc/*.hip $P/csrc/*.cpp; do
  b=$(basename $f)
  if [ "$b" = "$base" ]; then
    /opt/rocm/bin/hipcc $FLAGS "$@" -c $src -o $out/$b.o
    objs="$objs $out/$b.o"
  else
    objs="$objs $P/build/$b.o"
  fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/libafm.so $objs
echo $out/libafm.so
