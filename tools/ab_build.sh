#!/bin/bash
# Build libpggan_hip.so from a git revision's kernel sources into ab/lib_<name>.so
# (A/B timing of two builds in one GPU call: tools/kbench.py --lib ab/lib_<name>.so).
#   [AB_EXTRA=-DFOO=1] tools/ab_build.sh <name> [<rev>]     rev defaults to the working tree
set -e
cd "$(dirname "$0")/.."
name=$1; rev=${2:-}
tmp=$(mktemp -d)
mkdir -p "$tmp/pggan_amd/csrc" "$tmp/include" ab
if [ -n "$rev" ]; then
  for f in $(git ls-tree --name-only "$rev" pggan_amd/csrc/); do git show "$rev:$f" > "$tmp/$f"; done
  git show "$rev:include/pggan_hip.h" > "$tmp/include/pggan_hip.h"
else
  cp pggan_amd/csrc/*.hip pggan_amd/csrc/*.h pggan_amd/csrc/*.inc pggan_amd/csrc/Makefile "$tmp/pggan_amd/csrc/"
  cp include/pggan_hip.h "$tmp/include/"
fi
make -s -C "$tmp/pggan_amd/csrc" OUT="$(pwd)/ab/lib_$name.so" EXTRA="${AB_EXTRA:-}" -j2
rm -rf "$tmp"
echo "ab/lib_$name.so"
