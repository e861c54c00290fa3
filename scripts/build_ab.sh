#!/bin/bash
# A/B library variant: abvar/<name>.so = libspk_codec.so with the listed
# translation units rebuilt under extra -D flags (the bench / tests pick it up
# through SPK_CODEC_LIB=abvar/<name>.so).
# Usage: scripts/build_ab.sh name unit.hip[,unit2.hip] -DFOO=1 ...
set -e
cd "$(dirname "$0")/.."
name=$1; unit=$2; shift 2
mkdir -p abvar
objs=""
for s in spk_api spk_fixed spk_var spk_synth spk_nested spk_route; do
  if [[ ",$unit," == *",$s.hip,"* ]]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function \
      -I include "$@" -c yalantinglibs_amd/csrc/$s.hip -o abvar/${name}_$s.o
    objs="$objs abvar/${name}_$s.o"
  else
    objs="$objs yalantinglibs_amd/csrc/$s.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abvar/$name.so $objs
echo abvar/$name.so
