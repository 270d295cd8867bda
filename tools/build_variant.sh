#!/bin/bash
# Diagnostic / A-B builds: recompile ONE source with extra flags and link it with
# the release objects into irc_amd/lib/variants/<name>.so (load via IRC_LIB_PATH).
#   tools/build_variant.sh <name> <source.hip> <flags...>
set -e
name=$1; src=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/information-retrieval-with-contrastive-learning_amd/csrc
OBJ=$ROOT/build/obj
VO=$ROOT/build/obj_var/$name
mkdir -p "$VO" "$ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants"
make -s -C "$CS" -j8 >/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$ROOT/include" -I"$CS" \
  -munsafe-fp-atomics "$@" -c "$CS/$src" -o "$VO/${src%.hip}.o"
objs=$(ls $OBJ/*.o | grep -v "/${src%.hip}.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o \
  "$ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/$name.so" $objs "$VO/${src%.hip}.o"
echo "built variants/$name.so"
