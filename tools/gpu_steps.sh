#!/bin/bash
# Run GPU steps one after another, each under its own time limit, output to gpurun_out/<name>.txt.
# A step that ends with 0 or 1 (a test failure) lets the next one start; a fault, abort, segfault
# or time limit (anything else) ends the script there.
# usage: tools/gpu_steps.sh name1 secs1 'cmd1' name2 secs2 'cmd2' ...
mkdir -p gpurun_out
while [ $# -ge 3 ]; do
    name=$1; secs=$2; cmd=$3; shift 3
    echo "== $name ($secs s): $cmd"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.txt" 2>&1
    rc=$?
    echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.txt"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "== stopping after $name (rc=$rc)"; exit $rc; fi
done
