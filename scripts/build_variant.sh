#!/bin/bash
# build_variant.sh NAME "-DFLAGS..." : an alternative libspk_codec build under build_var/NAME.so
set -e
cd "$(dirname "$0")/.."
mkdir -p build_var/$1
objs=""
for s in spk_api spk_fixed spk_var spk_synth spk_nested spk_route; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function $2 -I include -c yalantinglibs_amd/csrc/$s.hip -o build_var/$1/$s.o &
  objs="$objs build_var/$1/$s.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build_var/$1.so $objs
