#!/bin/bash
# A/B builds of libdccrgx.so: tools/ab_build.sh NAME -DMACRO=VALUE ... builds
# tools/ab/libNAME.so from the current sources with the extra defines applied
# to one source (AB_SRC, default gol; the other objects from the library's own
# build in dccrg_amd/csrc/_build, which is left alone)
set -e
name=$1; shift
cd "$(dirname "$0")/../dccrg_amd/csrc"
mkdir -p ../../tools/ab/_build_$name
objs=""
for f in core grid halo gol golh scan sfc nbr explicit advect poisson amr amr_dev checkpoint stencil hybrid; do
  if [ "$f" = "${AB_SRC:-gol}" ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -munsafe-fp-atomics "$@" -c $f.hip -o ../../tools/ab/_build_$name/$f.o
    objs="$objs ../../tools/ab/_build_$name/$f.o"
  else
    objs="$objs _build/$f.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/ab/lib$name.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf ../../tools/ab/_build_$name
echo "tools/ab/lib$name.so"
