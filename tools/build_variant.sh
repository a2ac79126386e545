#!/bin/bash
# Build a variant of the library with extra compile flags for the fqz decoder,
# e.g. tools/build_variant.sh probe -DFQZ5_DEC_PROBE
# -> tools/variants/libfqz5_probe.so, loaded when FQZ5_LIB_VARIANT points at it.
set -e
name=$1; shift
here=$(cd "$(dirname "$0")" && pwd)
src=$here/../fqzcomp5_amd/csrc
out=$here/variants
mkdir -p $out/$name
objs=""
for f in $src/build/*.o; do
  b=$(basename $f)
  if [ "$b" = "fqz_decode.o" ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall --offload-arch=gfx950 "$@" -c $src/fqz_decode.hip -o $out/$name/fqz_decode.o
    objs="$objs $out/$name/fqz_decode.o"
  else
    objs="$objs $f"
  fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/libfqz5_$name.so $objs
echo $out/libfqz5_$name.so
