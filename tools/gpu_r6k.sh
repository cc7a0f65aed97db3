#!/bin/bash
# reasm_scan diagnostics: kernel stats of timing-only variants (tools/reasm_probe.py)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/rk && export TMPDIR=/tmp
for n in ${LIBS:-base NOINS NOREC NOWALK NOINPL}; do
  if [ "$n" = base ]; then lib=udpdk_amd/libudpdk_amd.so; else lib=tools/var/$n.so; fi
  export UDPDK_LIB_OVERRIDE=$PWD/$lib
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rk/$n -o r -- python3 tools/reasm_probe.py > gpurun_out/rk/$n.log 2>&1 || exit $?
  echo "$n $(python3 -c "
import csv
print(' '.join(r['Name'].split('(')[0].replace('udpdk::','')[6:]+'='+str(round(float(r['AverageNs'])/1000,1)) for r in csv.DictReader(open('gpurun_out/rk/$n/r_kernel_stats.csv')) if 'reasm' in r['Name']))")"
done
