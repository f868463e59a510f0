# SV tile-kernel A/B on the GPU box: tests, config 2 with the register-tile and the per-gate LDS
# kernels, timing-only variants (AQC_SV_DEBUG), kernel stats.  Outputs under gpurun_out/.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sv_tests.log 2>&1
timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/sv_reg.json 2>gpurun_out/sv_reg.err
AQC_SV_TILE=lds timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/sv_lds.json 2>gpurun_out/sv_lds.err
if [ -n "$SV_DEBUG" ]; then
AQC_SV_DEBUG=nogates timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/sv_nogates.json 2>gpurun_out/sv_dbg.err
AQC_SV_DEBUG=nophases timeout -k 10 200 python3 tools/configs_bench.py --configs 2 > gpurun_out/sv_nophases.json 2>>gpurun_out/sv_dbg.err
fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ksv -o run -- python3 tools/configs_bench.py --configs 2 > /dev/null 2>gpurun_out/ksv.err
python3 tools/rocpd_stats.py gpurun_out/ksv/run_results.db > gpurun_out/sv_kernel_stats.csv
rm -rf gpurun_out/ksv
