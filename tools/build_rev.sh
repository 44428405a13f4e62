#!/bin/bash
# Build the library of a git revision (default HEAD) as the frozen variant
# "old" (dynamic3dgaussians_amd/lib/libgsplat_hip_old.so) for A/B timing
# against the working tree: GSPLAT_VARIANT=old loads it (same C ABI required).
set -e
rev=${1:-HEAD}
name=${2:-old}
repo=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$repo" worktree add --detach "$tmp" "$rev" > /dev/null
(cd "$tmp" && python -m dynamic3dgaussians_amd.build --force > /dev/null)
cp "$tmp/dynamic3dgaussians_amd/lib/libgsplat_hip.so" "$repo/dynamic3dgaussians_amd/lib/libgsplat_hip_$name.so"
git -C "$repo" worktree remove --force "$tmp"
echo "$repo/dynamic3dgaussians_amd/lib/libgsplat_hip_$name.so <- $(git -C "$repo" rev-parse --short "$rev")"
