#!/bin/bash
# Builds an EXPERIMENT variant of libark_ddgi.so from a patched copy of the sources
# (the product sources stay free of experiment switches): copies
# arkoserenderer_amd/csrc to build_variants/<name>, applies the sed expressions given
# (each "file:sed-expression"), checks every expression changed its file, and builds
# arkoserenderer_amd/lib_<name>/libark_ddgi.so (select it with ARK_DDGI_LIB=...).
# Usage: tools/variant_lib.sh <name> 'file:s/a/b/' ['file:s/c/d/' ...]
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/build_variants/$NAME
rm -rf "$SRC"; mkdir -p "$SRC"
cp -r "$ROOT/arkoserenderer_amd/csrc/." "$SRC/"
rm -rf "$SRC/build" "$SRC"/build_*
# (the sources' ../../include/*.h resolve to the repository's include/ from here)
for p in "$@"; do
  f=${p%%:*}; e=${p#*:}
  before=$(md5sum "$SRC/$f" | cut -d' ' -f1)
  sed -i "$e" "$SRC/$f"
  after=$(md5sum "$SRC/$f" | cut -d' ' -f1)
  [[ "$before" != "$after" ]] || { echo "variant $NAME: '$e' changed nothing in $f"; exit 1; }
done
make -C "$SRC" -j8 OUT="$ROOT/arkoserenderer_amd/lib_$NAME/libark_ddgi.so" BUILD=build > "$ROOT/build_variants/$NAME.log" 2>&1 || { tail -20 "$ROOT/build_variants/$NAME.log"; exit 1; }
echo "built arkoserenderer_amd/lib_$NAME/libark_ddgi.so"
