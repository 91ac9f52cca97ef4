#!/bin/bash
# Build libmpccbf.so of a git revision into mpc-cbf_amd/build/rev_<name>/ (A/B timing against the
# working tree: MPCCBF_LIB=mpc-cbf_amd/build/rev_<name>/libmpccbf.so python bench.py ...).
#   bash tools/build_rev.sh <rev> <name>
set -e
REV=$1
NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" mpc-cbf_amd include | tar -x -C "$T"
make -C "$T/mpc-cbf_amd" -j8 build/libmpccbf.so > /dev/null
mkdir -p "$ROOT/mpc-cbf_amd/build/rev_$NAME"
cp "$T/mpc-cbf_amd/build/libmpccbf.so" "$ROOT/mpc-cbf_amd/build/rev_$NAME/"
rm -rf "$T"
echo "built $REV -> mpc-cbf_amd/build/rev_$NAME/libmpccbf.so"
