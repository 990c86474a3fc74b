#!/bin/bash
# Build libmfnerf_hip.so from the csrc of git revision REV into mf-nerf_amd/csrc/var/NAME.so (git-ignored,
# shipped to the GPU box) for library A/B runs (tools/ab_libs.sh: LIBS="- mf-nerf_amd/csrc/var/NAME.so").
# REV "-" takes the working tree's csrc (uncommitted edits included); EXTRA adds compiler flags
# (e.g. EXTRA=-DMFN_PROBE=1: a timing probe build, results invalid).
#     bash tools/build_variant.sh HEAD r4
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
if [ "$REV" = "-" ]; then
  mkdir -p "$TMP/mf-nerf_amd/csrc" && cp -r "$ROOT/include" "$TMP/" && cp "$ROOT"/mf-nerf_amd/csrc/*.hip "$ROOT"/mf-nerf_amd/csrc/*.hpp "$ROOT"/mf-nerf_amd/csrc/*.cpp "$ROOT"/mf-nerf_amd/csrc/Makefile "$TMP/mf-nerf_amd/csrc/"
else
  git -C "$ROOT" archive "$REV" mf-nerf_amd/csrc include | tar -x -C "$TMP"
fi
make -C "$TMP/mf-nerf_amd/csrc" -j8 EXTRA="$EXTRA" >/dev/null
mkdir -p "$ROOT/mf-nerf_amd/csrc/var"
cp "$TMP/mf-nerf_amd/libmfnerf_hip.so" "$ROOT/mf-nerf_amd/csrc/var/$NAME.so"
rm -rf "$TMP"
echo "built mf-nerf_amd/csrc/var/$NAME.so from $REV"
