#!/bin/bash
# Build the library from csrc/ with some files taken from a git revision, into
# tools/exp/variant_<name>/libwireglider_amd.so (for tools/ab_builds.sh).
# usage: [EXTRA_FLAGS=-D...] tools/build_variant.sh <name> <rev> <csrc file>...
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=$2; shift 2
SRC=$(mktemp -d); OUT=$ROOT/tools/exp/variant_$NAME; mkdir -p "$OUT"
cp "$ROOT"/wireglider_amd/csrc/* "$SRC"/
for f in "$@"; do git -C "$ROOT" show "$REV:wireglider_amd/csrc/$f" > "$SRC/$f"; done
objs=()
for s in "$SRC"/*.hip "$SRC"/*.cpp; do
  o=$SRC/$(basename "$s").o
  FF=""
  [ "$(basename "$s")" = aead.hip ] && FF="-mllvm -amdgpu-sched-strategy=max-ilp"  # wireglider_amd/_build.py FILE_FLAGS
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -Wno-unused-function ${EXTRA_FLAGS:-} $FF -I"$ROOT/include" -I"$SRC" \
    -x hip -c "$s" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libwireglider_amd.so" "${objs[@]}" -lpthread
rm -rf "$SRC"
echo "$OUT/libwireglider_amd.so"
