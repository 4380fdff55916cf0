#!/bin/bash
# Build libdhcos.so from a git revision (default HEAD) into dhcos/libdhcos_base.so for A/B runs.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD}
W=$(mktemp -d /tmp/dhcos_base.XXXX)
git -C "$ROOT" worktree add -q --detach "$W" "$REV"
make -s -C "$W/option-pricing-ffn-lbfgs_amd/csrc" "$W/option-pricing-ffn-lbfgs_amd/dhcos/libdhcos.so"
cp "$W/option-pricing-ffn-lbfgs_amd/dhcos/libdhcos.so" "$ROOT/option-pricing-ffn-lbfgs_amd/dhcos/libdhcos_base.so"
git -C "$ROOT" worktree remove --force "$W"
echo "built libdhcos_base.so from $(git -C "$ROOT" rev-parse --short "$REV")"
