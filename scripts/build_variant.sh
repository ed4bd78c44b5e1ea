#!/bin/bash
# Builds a variant of libmsl_hip.so for a same-box A/B (scripts/gpu_ab.sh): the csrc/ and include/ trees are
# copied to /tmp, each sed expression is applied to the named source file, and the library is built there and
# copied to maxsquareloss_amd/_lib/<tag>/libmsl_hip.so (git-ignored; it travels to the GPU box).
#   scripts/build_variant.sh <tag> [<file> <sed expression>]...
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; shift
T=/tmp/msl_var/$TAG
rm -rf "$T" && mkdir -p "$T/maxsquareloss_amd" "$T/maxsquareloss_amd/_lib"
cp -r "$R/include" "$T/include"
cp -r "$R/maxsquareloss_amd/csrc" "$T/maxsquareloss_amd/csrc"
while [ $# -ge 2 ]; do
  f=$T/maxsquareloss_amd/csrc/$1
  before=$(md5sum "$f")
  sed -i -e "$2" "$f"
  [ "$before" != "$(md5sum "$f")" ] || { echo "sed '$2' changed nothing in $1" >&2; exit 1; }
  shift 2
done
make -s -C "$T/maxsquareloss_amd/csrc" -j8 >/dev/null
mkdir -p "$R/maxsquareloss_amd/_lib/$TAG"
cp "$T/maxsquareloss_amd/_lib/libmsl_hip.so" "$R/maxsquareloss_amd/_lib/$TAG/libmsl_hip.so"
echo "built maxsquareloss_amd/_lib/$TAG/libmsl_hip.so"
