#!/bin/bash
# round-6 GPU call: STAGES (space-separated) from suite | smoke | bench | launch2 | c3 | prof
#   suite  : the whole -m gpu suite (one pytest process)      -> gpurun_out/r6_${TAG}_suite.log
#   smoke  : __graft_entry__.smoke()
#   bench  : the default bench line (driver's command)          -> gpurun_out/r6_${TAG}_bench.{json,err}
#   launch2: `python bench.py --gpus 2` (gloo, one GPU: the self-launcher)
#   c3     : C3 fp32 + C2 bf16 lines without CPU legs
#   prof   : rocprofv3 --kernel-trace --stats of the default C2 bench (+ C3 fp32 extra)
#   ab     : env A/B (tools/gpu_ab_env.sh "$AB" "$AB_CFGS")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-a}
for s in ${STAGES:-suite smoke bench}; do
  echo "[gpu_r6] stage $s ($(date +%T))"
  case $s in
    suite) timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread \
             -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/r6_${TAG}_suite.log 2>&1; rc=$?
           tail -4 gpurun_out/r6_${TAG}_suite.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_${TAG}_smoke.log 2>&1; rc=$?
           tail -2 gpurun_out/r6_${TAG}_smoke.log ;;
    bench) timeout -k 10 900 python -u bench.py > gpurun_out/r6_${TAG}_bench.json 2> gpurun_out/r6_${TAG}_bench.err; rc=$?
           cut -c1-600 gpurun_out/r6_${TAG}_bench.json ;;
    launch2) RSYS_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --extra= \
             --no-cpu-baseline > gpurun_out/r6_${TAG}_launch2.json 2> gpurun_out/r6_${TAG}_launch2.err; rc=$?
           cut -c1-300 gpurun_out/r6_${TAG}_launch2.json ;;
    c3) timeout -k 10 400 python -u bench.py --config c3 --dtype fp32 --steps ${STEPS:-50} --no-cpu-baseline \
          --extra c2:bf16 > gpurun_out/r6_${TAG}_c3.json 2> gpurun_out/r6_${TAG}_c3.err; rc=$?
        python3 -c "
import json; d=json.loads(open('gpurun_out/r6_${TAG}_c3.json').read().strip().splitlines()[-1])
print('c3 fp32', d['ms_per_step'], 'c2 bf16', d['extra']['c2_bf16']['ms_per_step'])" ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
          timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_${TAG}_prof -o run -- \
            python3 bench.py --no-cpu-baseline --extra c3:fp32 --prof-markers > gpurun_out/r6_${TAG}_prof.log 2>&1; rc=$? ;;
    ab) REPS=${REPS:-2} timeout -k 10 900 bash tools/gpu_ab_env.sh "$AB" "${AB_CFGS:-c3:fp32 c2:bf16}"; rc=$? ;;
    *) echo "unknown stage $s"; rc=2 ;;
  esac
  [ $rc -eq 0 ] || { echo "[gpu_r6] stage $s failed rc=$rc"; exit $rc; }
done
