#!/bin/bash
# Round 6, second closing run: the whole GPU suite, then tools/r6_final.sh (bench line + rocprofv3
# stats + PMC + FETCH traffic + smoke) on the final product.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r6_suite.sh || exit $?
bash tools/r6_final.sh
