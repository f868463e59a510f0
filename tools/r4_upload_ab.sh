#!/bin/bash
# Round-4 call: upload threshold A/B -- config 2 and single-state latency with the copy kernel
# from 16 KB (default), for every size (AQC_UPLOAD_MIN_KB=0) and never (AQC_UPLOAD=memcpy).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/upab_steps.txt
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/upab_steps.txt
  return $rc
}
for i in 1 2; do
  step ab_c2_16k_$i 200 python3 tools/configs_bench.py --configs 2 || exit $?
  AQC_UPLOAD_MIN_KB=0 step ab_c2_0k_$i 200 python3 tools/configs_bench.py --configs 2 || exit $?
  AQC_UPLOAD=memcpy step ab_c2_memcpy_$i 200 python3 tools/configs_bench.py --configs 2 || exit $?
done
step ab_lat_16k 300 python3 tools/latency_probe.py || exit $?
AQC_UPLOAD_MIN_KB=0 step ab_lat_0k 300 python3 tools/latency_probe.py || exit $?
AQC_UPLOAD=memcpy step ab_lat_memcpy 300 python3 tools/latency_probe.py || exit $?
step ab_roto_16k 300 python3 tools/roto_profile.py || exit $?
