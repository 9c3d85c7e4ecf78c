#!/bin/bash
# SQ counters of the ranged table-gradient kernel (tools/range_one.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/pmcrange
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  ( cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d $ROOT/gpurun_out/pmcrange/s$i -o run --output-format csv -- python3 $ROOT/tools/range_one.py 2 ) > gpurun_out/pmcrange/s$i.log 2>&1
  rc=$?; echo "set $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, re
for f in sorted(glob.glob('gpurun_out/pmcrange/s*/run_counter_collection.csv')):
    agg = {}
    for r in csv.DictReader(open(f)):
        if 'range_kernel' in r['Kernel_Name']:
            agg.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
    for k, v in agg.items():
        print(f'{k:24s} {sum(v) / 2:16.0f}')
PY
