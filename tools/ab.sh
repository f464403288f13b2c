#!/usr/bin/env bash
# Interleaved A/B of gemm_tune specs: each spec timed R times in alternation (min reported by
# the reader).  Usage: AB_R=3 bash tools/ab.sh [--step] spec1 spec2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEP=""; if [ "$1" = "--step" ]; then STEP="--step"; shift; fi
A=""
for r in $(seq ${AB_R:-3}); do for s in "$@"; do A="$A $s"; done; done
timeout -k 10 500 python tools/gemm_tune.py ${AB_LIB:+--lib=$AB_LIB} $STEP $A 2>&1 | grep kernel_us | python3 -c "
import sys, collections
d = collections.OrderedDict()
for l in sys.stdin:
    k, v = l.split()[0], float(l.split('kernel_us=')[1].split()[0])
    d.setdefault(k, []).append(v)
for k, v in d.items(): print(f'{k:60s} min={min(v):7.2f} med={sorted(v)[len(v)//2]:7.2f} all={v}')
"
