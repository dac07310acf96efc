#!/bin/bash
# Run a GPU command on a frozen copy of the tree: gpurun uploads /root/repo
# when its call leaves the queue (minutes after it is made), so edits made
# meanwhile would land in the run.  This copies the tree as it is now (built
# libraries included; .git, gpurun_out and old stages left out) into .stage/,
# and runs the command there on the box.
# usage: tools/gpurun_staged.sh <timeout-seconds> '<command>'
#        (KEEP_STAGE=1: reuse the existing .stage, e.g. to retry a call that found no box)
set -u
cd "$(dirname "$0")/.."
T=$1; shift
CMD=$1
if [ "${KEEP_STAGE:-0}" != 1 ]; then
  rm -rf .stage && mkdir -p .stage
  tar --exclude=./.git --exclude=./gpurun_out --exclude=./.stage --exclude='*.o' --exclude='__pycache__' \
      --exclude='./ringpop_amd/build' --exclude='./ringpop_amd/build_diag' -cf - . | tar -C .stage -xf -
fi
# (the stage's gpurun_out is a link to the top-level one: gpurun watches and
# merges that directory, and a run writing only elsewhere looks hung)
exec /usr/local/graft/bin/gpurun --timeout "$T" -- "mkdir -p gpurun_out && rm -rf .stage/gpurun_out && ln -s ../gpurun_out .stage/gpurun_out && cd .stage && $CMD"
