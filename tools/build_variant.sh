#!/bin/bash
# Build an A/B variant of the product library from HEAD's working tree plus
# patches (tools only; the product is priskv_amd/lib/libpriskv_crc.so).
#
#   tools/build_variant.sh NAME [PATCH ...] [-D MACRO=V ...]
#
# Copies priskv_amd/csrc and include/ to a scratch tree, applies each PATCH
# (git apply, paths relative to the repo root), compiles with the extra
# -D flags, and leaves abbuild/NAME/libpriskv_crc.so for tools/ab_libs.py.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME="$1"; shift
TMP="$(mktemp -d /tmp/prv_variant.XXXXXX)"
trap 'rm -rf "$TMP"' EXIT
mkdir -p "$TMP/priskv_amd" "$TMP/include"
cp -r "$ROOT/priskv_amd/csrc" "$TMP/priskv_amd/"
cp "$ROOT"/include/*.h "$TMP/include/"
rm -f "$TMP"/priskv_amd/csrc/*.o
DEFS=""
while [ $# -gt 0 ]; do
  case "$1" in
    -D) DEFS="$DEFS -D$2"; shift 2 ;;
    *) (cd "$TMP" && git apply "$ROOT/$1"); shift ;;
  esac
done
make -s -C "$TMP/priskv_amd/csrc" HIPFLAGS_EXTRA="$DEFS" ../lib/libpriskv_crc.so
mkdir -p "$ROOT/abbuild/$NAME"
cp "$TMP/priskv_amd/lib/libpriskv_crc.so" "$ROOT/abbuild/$NAME/"
echo "abbuild/$NAME/libpriskv_crc.so"
