#!/bin/bash
# Build a variant of the library with extra compile flags for one source,
# e.g. tools/build_variant.sh probe fqz_decode -DFQZ5_DEC_PROBE
#      tools/build_variant.sh cprobe rans_chain -DFQZ5_CHAIN_PROBE
# -> tools/variants/libfqz5_<name>.so, loaded when FQZ5_LIB_VARIANT points at it.
set -e
name=$1; shift
srcname=$1; shift
here=$(cd "$(dirname "$0")" && pwd)
src=$here/../fqzcomp5_amd/csrc
out=${VARIANT_DIR:-$here/variants}
mkdir -p $out/$name
objs=""
for f in $src/build/*.o; do
  b=$(basename $f)
  if [ "$b" = "$srcname.o" ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall --offload-arch=gfx950 "$@" -c $src/$srcname.hip -o $out/$name/$srcname.o
    objs="$objs $out/$name/$srcname.o"
  else
    objs="$objs $f"
  fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/libfqz5_$name.so $objs
echo $out/libfqz5_$name.so
