#!/bin/bash
# Runs one GPU step under a time limit: `tools/gpu_step.sh SECONDS OUT -- cmd ...`
# (stdout -> OUT, stderr -> OUT.err).  Exit 0 when the command ended by
# itself with status 0 or 1 (1: failed tests — later steps may still run);
# any other status (a fault, an abort, a time limit) is returned, so that
# `gpu_step ... && gpu_step ...` chains stop there.
t=$1; out=$2; shift 3
mkdir -p "$(dirname "$out")"
timeout -k 10 "$t" "$@" > "$out" 2> "$out.err"
rc=$?
echo "[gpu_step] rc=$rc: $*" >> "$out.err"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then exit 0; fi
echo "[gpu_step] stopping: rc=$rc ($*)"; tail -20 "$out.err"; exit $rc
