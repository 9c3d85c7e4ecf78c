#!/bin/bash
# Round profile set: C2 and C3, each a rocprofv3 kernel-trace summary plus FETCH_SIZE / WRITE_SIZE
# --pmc passes bracketing one entry point (tools/gpu_prof.sh); outputs in gpurun_out/prof_<tag>/.
# Usage: tools/gpu_prof_all.sh "tag|bracket|bench args[|notrace]" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for spec in "$@"; do
  IFS="|" read -r tag bracket args notrace <<< "$spec"
  rm -rf gpurun_out/prof
  PMC=1 NOTRACE=$notrace BRACKET=$bracket BENCH_ARGS="$args" bash tools/gpu_prof.sh || exit 1
  rm -rf gpurun_out/prof_$tag && mv gpurun_out/prof gpurun_out/prof_$tag
  rm -rf gpurun_out/prof_$tag/trace
done
