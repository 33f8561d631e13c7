#!/bin/bash
# Build libhsflow.so of another git revision into cpp-optical-flow_amd/lab/
# (same-box A/Bs with scripts/lab/k4_variants.py probe):
#   bash scripts/lab/build_rev.sh REV NAME   ->  lab/libhsflow_NAME.so
set -e
rev=${1:?revision}; name=${2:?name}
root=$(cd "$(dirname "$0")/../.." && pwd)
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
git -C "$root" archive "$rev" cpp-optical-flow_amd include | tar -x -C "$tmp"
make -s -C "$tmp/cpp-optical-flow_amd" -j8 libhsflow.so
mkdir -p "$root/cpp-optical-flow_amd/lab"
cp "$tmp/cpp-optical-flow_amd/libhsflow.so" "$root/cpp-optical-flow_amd/lab/libhsflow_$name.so"
echo "built lab/libhsflow_$name.so from $rev"
