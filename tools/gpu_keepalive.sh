#!/bin/bash
# Runs "$@" with a line appended to gpurun_out/alive.txt every 50 s, so a long
# quiet step (a big oracle comparison) is not taken for a hung GPU command.
mkdir -p gpurun_out
( while sleep 50; do date +%T >> gpurun_out/alive.txt; done ) &
KP=$!
"$@"
rc=$?
kill $KP 2>/dev/null
exit $rc
