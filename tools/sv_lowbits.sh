set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sv_tests.log 2>&1
for c in 0 1 2 3 4; do
AQC_SV_LOWBITS=$c timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/sv_low$c.json 2>gpurun_out/sv_low.err
AQC_SV_LOWBITS=$c AQC_SV_DEBUG=nophases timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/sv_lownp$c.json 2>gpurun_out/sv_low.err
done
