#!/bin/bash
# A/B tooling: build the library from another git revision (or with one file from it) into
# ab_libs/<name>.so for tools/with_lib.py, leaving the in-tree build alone.
#   bash tools/build_ab.sh <name> <rev> [file under dialog_amd/csrc ...]
# (no files: the whole dialog_amd/csrc + include at <rev>; files: the working tree with those
# files taken from <rev>)
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; rev=$2; shift 2
tmp=$(mktemp -d)
cp -r dialog_amd include "$tmp/"
rm -rf "$tmp/dialog_amd/build" "$tmp/dialog_amd/libdialog_amd.so"
if [ $# -eq 0 ]; then
  for f in $(git ls-tree -r --name-only "$rev" dialog_amd/csrc include); do git show "$rev:$f" > "$tmp/$f"; done
else
  for f in "$@"; do git show "$rev:dialog_amd/csrc/$f" > "$tmp/dialog_amd/csrc/$f"; done
fi
(cd "$tmp" && python3 -c "import sys; sys.path.insert(0, '.'); from dialog_amd import build as B; B.build(force=True)")
mkdir -p ab_libs
cp "$tmp/dialog_amd/libdialog_amd.so" "ab_libs/$name.so"
rm -rf "$tmp"
echo "ab_libs/$name.so"
