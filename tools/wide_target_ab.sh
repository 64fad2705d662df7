#!/bin/bash
# Whole-step A/B of the wide weight gradients' pixel-split target (256 default: two slabs and
# a reduction launch at 512 channels; 128: one split, direct accumulation, half the CUs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ENV_AB=PG_WG_TARGET_WIDE AB_VALS="256 128" AB_SPECS="w:32:512:512:0 w:64:512:512:0 w:128:256:512:1 w:256:128:256:1" timeout -k 10 300 bash tools/env_ab.sh 2 || exit 1
timeout -k 10 900 bash tools/ab_env.sh 2 "e:PG_WG_TARGET_WIDE=256" "e:PG_WG_TARGET_WIDE=128" "e:PG_WG_TARGET_WIDE=64"
