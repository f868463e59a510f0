#!/bin/bash
# Round-4 call: the copy-kernel uploads everywhere (aqc::upload_async) -- the whole GPU suite, then
# latency (single evaluations, Rotoselect gate) and config 2 with the kernel uploads and with
# AQC_UPLOAD=memcpy (A/B), then the bench step (no CPU baseline).  Any failure ends it.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/upload_steps.txt
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/upload_steps.txt
  return $rc
}
step usuite 700 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
step lat_kernel 300 python3 tools/latency_probe.py || exit $?
AQC_UPLOAD=memcpy step lat_memcpy 300 python3 tools/latency_probe.py || exit $?
step roto_kernel 300 python3 tools/roto_profile.py || exit $?
AQC_UPLOAD=memcpy step roto_memcpy 300 python3 tools/roto_profile.py || exit $?
step c2_kernel 200 python3 tools/configs_bench.py --configs 2,4 || exit $?
AQC_UPLOAD=memcpy step c2_memcpy 200 python3 tools/configs_bench.py --configs 2,4 || exit $?
step ubench 400 python3 bench.py --no-cpu-baseline || exit $?
