#!/bin/bash
# Sweep of tools/ubench/mem_pattern over modes, waves per CU, store policy, XCD remap.
set -eu -o pipefail
B=${GRAFT_REPO_ROOT:-$(pwd)}/tools/ubench/mem_pattern
for m in 0 3; do for w in 8 12; do for nt in 0 1; do for x in 0 1; do
  timeout -k 5 30 "$B" $m $w $nt $x
done; done; done; done
