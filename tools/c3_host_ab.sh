#!/bin/bash
# Same-box A/B of the host-pointer C3 round (tools/c3_host_probe.py) over
# process-level switches: ENVS="name=VAR=val[;VAR=val] ..." alternated REPS
# times, each in its own process (stream kinds are fixed per process), with
# C3_PROBE_CONFIGS passed through.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for kv in $ENVS; do
    name=${kv%%=*}; envs=${kv#*=}
    ( IFS=';'; for e in $envs; do export "$e"; done
      timeout -k 10 200 python tools/c3_host_probe.py ${CALLS:-10} > gpurun_out/c3ab_$name.jsonl 2> gpurun_out/c3ab_$name.err ) || exit 1
    sed "s/^/$name $rep /" gpurun_out/c3ab_$name.jsonl
  done
done
