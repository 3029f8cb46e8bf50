#!/bin/bash
# Kernel-time A/B of two builds of the HIP library: rocprofv3 kernel stats of bench.py (2 timed
# steps) with the in-tree library and with $B (SYSML_HIP_LIB), top kernels of each.
R=$GRAFT_REPO_ROOT
B=${B:-$R/systemml_amd/ops/lib/ab/libsysml_hip_base.so}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
for V in new base; do
  if [ $V = base ]; then export SYSML_HIP_LIB=$B; else unset SYSML_HIP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kab_$V -o run --output-format csv -- \
      python3 $R/bench.py --steps 2 --warmup 1 "$@" > $R/gpurun_out/kab_$V.log 2>&1 || exit $?
  S=$(find $R/gpurun_out/kab_$V -name '*kernel_stats.csv' | head -1)
  echo "== $V"
  python3 - "$S" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:6]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} calls avg {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:70]}')
PY
done
