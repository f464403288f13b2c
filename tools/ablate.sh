#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for a in 0 1 2 4 8 6 9 15; do
  GQ_ABLATE=$a timeout -k 10 120 python tools/ablate.py ${1:-q8_0_4096x4096_m128} 2>&1 | grep ablate= || exit 1
done
