#!/bin/bash
# Cost split of the sign-bit input-gradient conv (X_BITS | MASK | UPS_IN) at 1024^2 / 512^2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 200 python tools/kbench.py --iters 30 c:1024:32:16:521 c:1024:32:16:9 c:1024:32:16:1 c:1024:32:16:0 c:1024:16:16:8 c:1024:16:16:0 c:512:64:32:521 c:512:64:32:9 c:512:64:32:1 c:512:64:32:0 2>&1 | grep -v amdgpu
