#!/bin/bash
# The steps of one gpurun call, each under its own time limit, stopping at
# the first failure (a step that faults, aborts or times out ends the call:
# nothing more runs on the GPU after it).
#
#   gpurun -- 'bash scripts/gpu_steps.sh OUT "name|seconds|command" ...'
#
# OUT is a directory under gpurun_out/; step `name` writes OUT/name.log; in a
# command @OUT@ stands for that directory and @ROOT@ for the repo root.  A
# command runs from the repo root; one that profiles puts `cd /tmp && export
# TMPDIR=/tmp &&` first and the program itself right after rocprofv3's `--`.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
out=$GRAFT_REPO_ROOT/gpurun_out/$1
shift
mkdir -p "$out"
export PYTHONUNBUFFERED=1 OUT="$out"
i=0
for step in "$@"; do
  i=$((i + 1))
  name=${step%%|*}
  rest=${step#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  cmd=${cmd//@OUT@/$out}
  cmd=${cmd//@ROOT@/$GRAFT_REPO_ROOT}
  echo "[$i] $name (limit $secs s): $cmd"
  (cd "$GRAFT_REPO_ROOT" && timeout -k 10 "$secs" bash -c "$cmd") > "$out/$name.log" 2>&1
  rc=$?
  echo "[$i] $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
echo done
