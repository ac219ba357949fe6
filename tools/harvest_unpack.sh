#!/usr/bin/env bash
# Replace warpdb_amd/.kernel_cache with the objects a harvest run packed
# (tools/harvest_kernel_cache.sh).  usage: bash tools/harvest_unpack.sh TAG
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
T=$R/gpurun_out/${1:-harvest}/kernel_cache.tgz
test -s "$T"
rm -rf "$R/warpdb_amd/.kernel_cache"
mkdir -p "$R/warpdb_amd/.kernel_cache"
tar xzf "$T" -C "$R/warpdb_amd/.kernel_cache"
ls "$R/warpdb_amd/.kernel_cache" | wc -l
