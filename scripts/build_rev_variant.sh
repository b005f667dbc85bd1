#!/bin/bash
# Build the library of a git revision into fabric-token-sdk_amd/zkatdlog/_lib/ab/
# libftsamd_<name>.so for a same-box A/B against the working tree (ab_lib.sh).
#   bash scripts/build_rev_variant.sh <rev> <name>
set -eu
cd "$(dirname "$0")/.."
rev=$1; name=$2
wt=/tmp/fts_wt_$name
rm -rf "$wt"; git worktree prune
git worktree add -f --detach "$wt" "$rev" > /dev/null
mkdir -p "$wt/fabric-token-sdk_amd/build"
# reuse this tree's objects as a starting point: build.py recompiles what changed by mtime
python3 "$wt/fabric-token-sdk_amd/build.py" -j 8 > /dev/null
mkdir -p fabric-token-sdk_amd/zkatdlog/_lib/ab
cp "$wt/fabric-token-sdk_amd/zkatdlog/_lib/libftsamd.so" fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_$name.so
git worktree remove --force "$wt"
echo "built fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_$name.so from $(git rev-parse --short $rev)"
