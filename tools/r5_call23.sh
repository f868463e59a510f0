#!/bin/bash
# Round-5 GPU call 23: config 5 in-process after configs 2 / 4 ran 0.365 ms per gate against 0.29
# alone -- the two-stage schedule's four streams sharing the process's four hardware queues with the
# earlier configs' streams?  Config 5 alone, after config 2, after 2 and 4 with GPU_MAX_HW_QUEUES=8,
# and the same with the schedule on three streams (eigenpairs on the compact-WY stream: libaqchip_3s.so).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/adaptaqc_amd
run() {  # tag lib configs [env]
  local t=$1 lib=$2 c=$3; shift 3
  env "$@" AQC_LIB=$lib timeout -k 10 300 python3 tools/configs_bench.py --configs $c > gpurun_out/r5c23_$t.json 2> gpurun_out/r5c23_$t.err || exit $?
}
run cur_5 $L/libaqchip.so 5
run cur_25 $L/libaqchip.so 2,5
run cur_245 $L/libaqchip.so 2,4,5
run cur_245_q8 $L/libaqchip.so 2,4,5 GPU_MAX_HW_QUEUES=8
run s3_5 $L/libaqchip_3s.so 5
run s3_245 $L/libaqchip_3s.so 2,4,5
exit 0
