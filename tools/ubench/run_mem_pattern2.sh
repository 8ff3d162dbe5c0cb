#!/bin/bash
# mem_pattern: stores spread between VALU work vs burst after it (modes 4/5)
set -eu -o pipefail
B=${GRAFT_REPO_ROOT:-$(pwd)}/tools/ubench/mem_pattern
timeout -k 5 30 "$B" 0 12 1 1
for w in 1 2 4; do for m in 4 5; do
  timeout -k 5 30 "$B" $m 12 1 1 $w
done; done
