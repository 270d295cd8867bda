#!/bin/bash
# Diagnostic / A-B builds: recompile the given sources with extra flags and link
# them with the release objects into irc_amd/lib/variants/<name>.so (load via
# IRC_LIB_PATH).
#   tools/build_variant.sh <name> "<source.hip> [more.hip ...]" <flags...>
set -e
name=$1; srcs=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/information-retrieval-with-contrastive-learning_amd/csrc
OBJ=$ROOT/build/obj
VO=$ROOT/build/obj_var/$name
mkdir -p "$VO" "$ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants"
make -s -C "$CS" -j8 >/dev/null
objs=$(ls $OBJ/*.o)
for src in $srcs; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$ROOT/include" -I"$CS" \
    -munsafe-fp-atomics "$@" -c "$CS/$src" -o "$VO/${src%.hip}.o" &
  objs=$(echo "$objs" | grep -v "/${src%.hip}.o$")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o \
  "$ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/$name.so" $objs $VO/*.o
echo "built variants/$name.so"
