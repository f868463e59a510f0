set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SKIP_TESTS=1 ROUND=r3 bash tools/profile_round.sh
L=$PWD/adaptaqc_amd/libaqchip_it2.so
AQC_LIB=$L timeout -k 10 120 python3 tools/svd32_probe.py 3 > gpurun_out/ab_probe_it2.txt 2>&1
timeout -k 10 120 python3 tools/svd32_probe.py 3 > gpurun_out/ab_probe_cur.txt 2>&1
AQC_LIB=$L timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_it2.log 2>&1
rm -f gpurun_out/abr_*
AB_REPS=2 timeout -k 10 300 bash tools/ab_repeat.sh cur it2
