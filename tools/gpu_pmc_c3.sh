#!/bin/bash
# re-collect the C3 tower-backward PMC traffic (fp32 and bf16) after a tower change
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
for dt in fp32 bf16; do
  mkdir -p gpurun_out/pmc_$dt
  for ctr in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -d $ROOT/gpurun_out/pmc_$dt/pmc_$ctr -o run --output-format csv -- python3 $ROOT/bench.py --warmup 2 --pmc-bracket rs_tower_bwd --config c3 --dtype $dt ) > gpurun_out/pmc_$dt/pmc_$ctr.log 2>&1
    rc=$?; echo "$dt pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_traffic.py gpurun_out/pmc_$dt gpurun_out/pmc_$dt/pmc_FETCH_SIZE.log > gpurun_out/pmc_$dt/traffic.json 2> gpurun_out/pmc_$dt/traffic.err
  echo "$dt traffic rc=$?"; head -16 gpurun_out/pmc_$dt/traffic.json
done
