#!/bin/bash
# Build librti.so from a git revision into ab/<name>/ for same-box A/B timing (measurement only):
#   tools/ab_build.sh <rev> <name>   ->  RTI_PKG_DIR=ab/<name>/smartphone-based-rti_amd python tools/...
set -e
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
dst=$root/ab/$name
rm -rf "$dst"; mkdir -p "$dst"
git -C "$root" archive "$rev" smartphone-based-rti_amd include | tar -x -C "$dst"
make -C "$dst/smartphone-based-rti_amd" -j8 >/dev/null
echo "built $rev -> $dst/smartphone-based-rti_amd/rti/librti.so"
