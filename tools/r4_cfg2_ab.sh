#!/bin/bash
# Round-4 call: config 2 with the plan uploaded by a copy kernel (default) and by hipMemcpyAsync
# (AQC_UPLOAD=memcpy), alternating, after the SV tests; then the device timeline of the default.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/cfg2ab_steps.txt
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/cfg2ab_steps.txt
  return $rc
}
step sv_tests 300 python3 -u -m pytest tests/test_gpu_sv.py -x -q --timeout 120 --timeout-method thread || exit $?
for i in 1 2; do
  step cfg2_kernel_$i 200 python3 tools/configs_bench.py --configs 2 || exit $?
  AQC_UPLOAD=memcpy step cfg2_memcpy_$i 200 python3 tools/configs_bench.py --configs 2 || exit $?
done
step tl2 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tl2 -o run -- python3 tools/configs_bench.py --configs 2 --reps 1 || exit $?
python3 tools/timeline_gaps.py gpurun_out/tl2/run > gpurun_out/cfg2_gaps_kernelcopy.json
rm -f gpurun_out/tl2/run_agent_info.csv
