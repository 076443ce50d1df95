#!/bin/bash
# Build libkp.so as it was at a git commit into tools/variants/<name>/libkp.so (A/B of kernel changes on one box:
# tools/gpu_ab_kernel.sh). usage: build_commit_variant.sh <name> <commit>
set -e
name=$1; commit=$2
root=$(cd "$(dirname "$0")/.." && pwd)
wt=/tmp/kp_wt_$name
rm -rf "$wt"; git -C "$root" worktree prune
git -C "$root" worktree add --detach "$wt" "$commit" > /dev/null
make -C "$wt/karpenter-provider-aws_amd" -j8 > /dev/null
mkdir -p "$root/tools/variants/$name"
cp "$wt/karpenter-provider-aws_amd/libkp.so" "$root/tools/variants/$name/libkp.so"
git -C "$root" worktree remove --force "$wt"
echo "built tools/variants/$name/libkp.so from $commit"
