#!/bin/bash
# Round 6, first GPU batch: the in-launch combine's tests + A/B (tools/r6_ilc.sh), then the 7B
# layer A/B against the round-4 tree (tools/r6_layer_ab.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r6_ilc.sh && bash tools/r6_layer_ab.sh
